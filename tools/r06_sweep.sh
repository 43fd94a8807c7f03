#!/bin/bash
# Round 6: the reference's published sweeps on MI355X (analysis/runner.py:99-192 and
# runner_maxspheres0.py:99-160 through tools/sweep.py), then a rocprofv3 kernel trace of the
# reference's default configuration (src/config.h:10-28: 800x600, 100 spheres, depth 3, M=0,
# 16 spp x 8 bounces) and of stats.csv:114's workload (1000 spheres, depth 5, M=1, 16 x 8, 1920x1080).
# usage (GPU box): bash tools/r06_sweep.sh OUTDIR [grids...]
set -eo pipefail
OUT=${1:-gpurun_out/r06/sweep}
shift || true
GRIDS=${*:-"runner maxspheres0"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
case "$OUT" in /*) ;; *) OUT="$R/$OUT" ;; esac
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for g in $GRIDS; do
  rm -f "$OUT/stats_$g.csv"
  timeout -k 10 1500 python3 -u "$R/tools/sweep.py" --grid "$g" --out "$OUT/stats_$g.csv" --timeout 120 \
    > "$OUT/sweep_$g.log" 2>&1
done
M="$R/build/ort_main"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o run -- \
  "$M" --spheres 100 --depth 3 --per-node 0 --samples 16 --bounces 8 --width 800 --height 600 --frames 20 --warmup 5 \
  > "$OUT/prof_default.log" 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_stats114" -o run -- \
  "$M" --spheres 1000 --depth 5 --per-node 1 --samples 16 --bounces 8 --width 1920 --height 1080 --frames 20 --warmup 5 \
  > "$OUT/prof_stats114.log" 2>&1
echo sweep done
