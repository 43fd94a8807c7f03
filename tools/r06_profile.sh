#!/bin/bash
# Runs ON the GPU box: tools/profile_box.sh for each config, summarised on the box
# (tools/summarize_profile.py) into gpurun_out/r06/sum/<config>.{md,json} + pmc_<config>.json,
# then the raw PMC CSVs (tens of MB each) are dropped so that gpurun_out stays under the copy-back
# limit.  usage: bash tools/r06_profile.sh "c3:20:20 c5:10:5 ref_default:20:20"
set -u
R=$(pwd)
mkdir -p gpurun_out/r06/sum
for spec in $1; do
  IFS=: read -r cfg steps warm <<< "$spec"
  tag=r06/prof_$cfg
  timeout -k 10 900 bash tools/profile_box.sh "$tag" "$cfg" "$steps" "$warm" || { echo "profile $cfg failed"; exit 1; }
  python3 tools/summarize_profile.py "gpurun_out/$tag" "gpurun_out/r06/sum/$cfg" "$cfg" > "gpurun_out/r06/sum/$cfg.log" 2>&1 \
    || { echo "summary $cfg failed"; cat "gpurun_out/r06/sum/$cfg.log"; exit 1; }
  rm -rf "gpurun_out/$tag"/pmc_*
  echo "summary $cfg ok"
done
du -ak gpurun_out | sort -n | tail -10
