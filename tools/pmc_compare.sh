#!/bin/bash
# Runs ON the GPU box: PMC passes over tools/prof_frame.py --both (packet and per-lane trace
# kernels in one run) -> gpurun_out/<tag>/pmc_<pass>/.  usage: tools/pmc_compare.sh <tag> [config]
set -u
TAG=${1:-cmp}
CFG=${2:-c3}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
run() {
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_$name -o pmc -- \
        python3 $R/tools/prof_frame.py --config $CFG --frames 2 --both > $OUT/pmc_$name.log 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then echo "pmc pass $name failed rc=$rc"; exit $rc; fi
}
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD
run b SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
run c SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC
run d SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM
echo "pmc $TAG done"
