#!/bin/bash
# Runs ON the GPU box: the device-side speculate / fall-back decision -- parity tests, then A/B
# against the host-side policy (build/ab/libdvA.so) static and with a turning camera, and the
# bench's moving-camera phase of config.h's default.
set -u
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_glsl_parity.py -m gpu -k "pixel or speculate or reference_shader or canonical" > gpurun_out/r06/spec3_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/r06/spec3_tests.log; exit 1; }
echo "tests ok"
B=build/ab
for c in ref_default ref_stats114; do
  timeout -k 10 300 python tools/ab_stream.py $B/libdvA.so $B/libdvB.so --config $c > gpurun_out/r06/ab_dev_$c.log 2>&1 || exit 1
  timeout -k 10 300 python tools/ab_stream.py $B/libdvA.so $B/libdvB.so --config $c --yaw-step 0.5 > gpurun_out/r06/ab_dev_${c}_moving.log 2>&1 || exit 1
done
timeout -k 10 300 python3 bench.py --config ref_default --no-cpu-baseline > gpurun_out/r06/bench_ref_default_dev.json 2> gpurun_out/r06/bench_ref_default_dev.err || exit 1
echo "ab ok"
