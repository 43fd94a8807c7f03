#!/bin/bash
# Runs ON the GPU box: SPEC with chunks of >= 4 samples -- parity tests, then option off/on A/B
# on the reference's frames and the small-scene rows the one-sample chunks had slowed.
set -u
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_glsl_parity.py -m gpu > gpurun_out/r06/spec2_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/r06/spec2_tests.log; exit 1; }
echo "tests ok"
A=octreeraytracer_amd/lib/libort_analysis.so
run() { name=$1; shift; timeout -k 10 300 python tools/ab_stream.py $A@pixel_speculate=0 $A --rounds 8 "$@" > gpurun_out/r06/ab_spec2_$name.log 2>&1 || { echo "ab $name failed"; tail -5 gpurun_out/r06/ab_spec2_$name.log; exit 1; }; }
run ref_default --config ref_default
run ref_stats114 --config ref_stats114
run small10_16x8_1080 --config c2 --spheres 10 --tree-depth 1 --samples 16 --max-depth 8
run small10_32x16_1080 --config c2 --spheres 10 --tree-depth 1 --samples 32 --max-depth 16
run small100_16x8_1080 --config c2 --spheres 100 --tree-depth 1 --samples 16 --max-depth 8
run c2_8x8 --config c2 --samples 8 --max-depth 8
echo "ab ok"
