#!/bin/bash
# Runs ON the GPU box: samples in parallel (ORT_OPT_PIXEL_SPECULATE) -- the parity tests, then
# option off/on A/B on the reference's frames and larger trees, static and with a turning camera.
set -u
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_glsl_parity.py tests/test_gpu_cost_order.py tests/test_gpu_async.py -m gpu > gpurun_out/r06/spec_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/r06/spec_tests.log; exit 1; }
echo "tests ok"
A=octreeraytracer_amd/lib/libort_analysis.so
run() { name=$1; shift; timeout -k 10 300 python tools/ab_stream.py $A@pixel_speculate=0 $A "$@" > gpurun_out/r06/ab_spec_$name.log 2>&1 || { echo "ab $name failed"; tail -5 gpurun_out/r06/ab_spec_$name.log; exit 1; }; }
run ref_default --config ref_default
run ref_default_moving --config ref_default --yaw-step 0.5
run ref_stats114 --config ref_stats114
run ref_stats114_moving --config ref_stats114 --yaw-step 0.5
run mid30k --config c2 --spheres 30000 --tree-depth 7 --samples 4 --max-depth 8
run runner10_32x16 --config ref_default --spheres 10 --tree-depth 1 --samples 32 --max-depth 16
echo "ab ok"
