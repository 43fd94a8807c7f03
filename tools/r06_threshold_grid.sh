#!/bin/bash
# Runs ON the GPU box: whole-pixel paths (heavy blocks first) against the per-bounce pipeline,
# 1080p, over trees of 1.5-11 M nodes x samples x bounces -- the data for the auto rule.
set -u
mkdir -p gpurun_out/r06/grid
A=octreeraytracer_amd/lib/libort_analysis.so
for tree in 30000:7 20000:8 50000:8 100000:8; do
  IFS=: read -r n d <<< "$tree"
  for sb in 2:4 3:5 4:4 2:8 4:8; do
    IFS=: read -r ns md <<< "$sb"
    timeout -k 10 300 python tools/ab_stream.py $A@pixel_paths=0 $A@pixel_paths=1 --rounds 4 --block 4 --config c2 \
      --spheres $n --tree-depth $d --samples $ns --max-depth $md > gpurun_out/r06/grid/${n}_d${d}_s${ns}x${md}.log 2>&1 || exit 1
    echo "$n d$d ${ns}x${md} $(grep -c 'x of' gpurun_out/r06/grid/${n}_d${d}_s${ns}x${md}.log)"
  done
done
