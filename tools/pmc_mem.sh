#!/bin/bash
# Runs ON the GPU box: vector-memory pipeline counters (TA address/data path, TD, per-CU L1)
# over tools/prof_frame.py, one rocprofv3 --pmc pass each (at most 2 TA_, 2 TD_, 4 TCP_ per
# pass) -> gpurun_out/<tag>/pmc_<pass>/.  Summarise with
#   python tools/summarize_profile.py gpurun_out/<tag> profiles/<name> <config> --no-record
# usage: tools/pmc_mem.sh <tag> [config]
set -u
TAG=${1:-mem}
CFG=${2:-c5}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
run() {
    local name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_$name -o pmc -- \
        python3 $R/tools/prof_frame.py --config $CFG --frames 2 --meta $OUT/meta.json > $OUT/pmc_$name.log 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then echo "pmc pass $name failed rc=$rc"; exit $rc; fi
    echo "pmc pass $name ok"
}
run ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD
run ta2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_LOAD_WAVEFRONTS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY
run td TD_TD_BUSY_sum TD_TC_STALL_sum SQ_INSTS_LDS SQ_ACTIVE_INST_LDS
run tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
echo "pmc mem $TAG done"
