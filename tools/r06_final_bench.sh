#!/bin/bash
# Runs ON the GPU box: the final build's bench lines (bench.py defaults per config) into
# gpurun_out/r06/final/bench_<config>.json, then the reference's sweeps (tools/r06_sweep.sh).
set -u
mkdir -p gpurun_out/r06/final
for c in c3 c5 ref_default ref_stats114 c2; do
  timeout -k 10 400 python3 -u bench.py --config $c > gpurun_out/r06/final/bench_$c.json 2> gpurun_out/r06/final/bench_$c.err \
    || { echo "bench $c failed"; tail -5 gpurun_out/r06/final/bench_$c.err; exit 1; }
  echo "bench $c ok"
done
[ "${1:-}" = "nosweep" ] && exit 0
bash tools/r06_sweep.sh gpurun_out/r06/sweep3 || { echo "sweep failed"; exit 1; }
