#!/bin/bash
# Runs ON the GPU box: whole-pixel paths (now with heavy blocks first) against the per-bounce
# pipeline on the trees around the auto rule's multi-sample limit (2^23 nodes).
set -u
mkdir -p gpurun_out/r06
A=octreeraytracer_amd/lib/libort_analysis.so
run() { name=$1; shift; timeout -k 10 300 python tools/ab_stream.py $A@pixel_paths=0 $A@pixel_paths=1 --rounds 6 --block 5 "$@" > gpurun_out/r06/thr2_$name.log 2>&1 || exit 1; }
run c3tree_s3d5 --config c2 --spheres 100000 --tree-depth 8 --samples 3 --max-depth 5
run c3tree_s4d8 --config c2 --spheres 100000 --tree-depth 8 --samples 4 --max-depth 8
run 50k_d8_s4d8 --config c2 --spheres 50000 --tree-depth 8 --samples 4 --max-depth 8
run 50k_d8_s2d4 --config c2 --spheres 50000 --tree-depth 8 --samples 2 --max-depth 4
