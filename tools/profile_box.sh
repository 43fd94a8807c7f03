#!/bin/bash
# Runs ON the GPU box (via gpurun): rocprofv3 kernel trace of bench.py plus separate PMC
# passes over tools/prof_frame.py.  Output under gpurun_out/<tag>/; summarise afterwards with
#   python tools/summarize_profile.py gpurun_out/<tag> profiles/<name> <config>
# usage: tools/profile_box.sh <tag> [config] [bench steps] [bench warmup]
# (C3 frames keep getting faster for the first ~15 frames of a run -- the clocks ramping up:
# profiles/r05_c3_warm3.md -- so short frames need a long warm-up for the summary to describe
# the steady state the bench line measures: c3 20 20)
set -u
TAG=${1:-prof}
CFG=${2:-c3}
STEPS=${3:-10}
WARM=${4:-3}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
run() {  # name, counters...  (each pass its own run; at most 8 SQ / 4 TCC / 2 GRBM counters)
    local name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_$name -o pmc -- \
        python3 $R/tools/prof_frame.py --config $CFG --frames 2 --meta $OUT/meta.json > $OUT/pmc_$name.log 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then echo "pmc pass $name failed rc=$rc"; exit $rc; fi
    echo "pmc pass $name ok"
}
# one frame in flight: each kernel alone on the GPU, as the roofline's kernel times in bench.py
# (its one-frame-in-flight phase when the default keeps two in flight)
echo "{\"steps\": $STEPS, \"warmup\": $WARM, \"config\": \"$CFG\", \"inflight\": 1}" > $OUT/bench_args.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
    python3 $R/bench.py --config $CFG --steps $STEPS --warmup $WARM --inflight 1 --no-cpu-baseline --moving-steps 0 > $OUT/trace_bench.log 2>&1 || { echo "trace failed"; exit 1; }
echo "kernel trace ok"
run fetch FETCH_SIZE
run write WRITE_SIZE
run valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM
run util SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT
run l2 TCC_HIT_sum TCC_MISS_sum
echo "profile $TAG done"
