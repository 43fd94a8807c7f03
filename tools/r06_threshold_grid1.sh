#!/bin/bash
# Runs ON the GPU box: as r06_threshold_grid.sh, one sample per pixel and deeper paths.
set -u
mkdir -p gpurun_out/r06/grid
A=octreeraytracer_amd/lib/libort_analysis.so
for tree in 10000:6 30000:7 100000:8; do
  IFS=: read -r n d <<< "$tree"
  for sb in 1:4 1:8 1:16 2:16; do
    IFS=: read -r ns md <<< "$sb"
    timeout -k 10 300 python tools/ab_stream.py $A@pixel_paths=0 $A@pixel_paths=1 --rounds 4 --block 4 --config c2 \
      --spheres $n --tree-depth $d --samples $ns --max-depth $md > gpurun_out/r06/grid/${n}_d${d}_s${ns}x${md}.log 2>&1 || exit 1
    echo "$n d$d ${ns}x${md} $(grep -c 'x of' gpurun_out/r06/grid/${n}_d${d}_s${ns}x${md}.log)"
  done
done
