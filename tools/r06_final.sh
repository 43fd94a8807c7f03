#!/bin/bash
# Runs ON the GPU box: the round's final checks -- every GPU test, smoke(), and the PMC profiles
# of the bench configs summarised into gpurun_out/r06/sum (tools/r06_profile.sh).
set -u
mkdir -p gpurun_out/r06/final
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/r06/final/gputest.log 2>&1 || { echo "gpu tests failed"; exit 1; }
echo "gpu tests ok"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/final/smoke.log 2>&1 \
  || { echo "smoke failed"; exit 1; }
echo "smoke ok"
bash tools/r06_profile.sh "${1:-c3:20:20 c5:10:5 ref_default:20:20 ref_stats114:10:5}"
