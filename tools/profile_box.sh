#!/bin/bash
# Runs ON the GPU box (via gpurun): rocprofv3 kernel trace of bench.py plus separate PMC
# passes over tools/prof_frame.py.  Output under gpurun_out/<tag>/.
# usage: tools/profile_box.sh <tag> [config]
set -u
TAG=${1:-prof}
CFG=${2:-c3}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
run() {  # name, counters...
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_$name -o pmc -- \
        python3 $R/tools/prof_frame.py --config $CFG --frames 2 > $OUT/pmc_$name.log 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then echo "pmc pass $name failed rc=$rc"; exit $rc; fi
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
    python3 $R/bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline > $OUT/trace_bench.log 2>&1 || { echo "trace failed"; exit 1; }
run fetch FETCH_SIZE
run write WRITE_SIZE
run ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
run ea2 TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum
run l2 TCC_HIT_sum TCC_MISS_sum
run valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM
run util SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
echo "profile $TAG done"
