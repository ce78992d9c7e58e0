#!/bin/bash
# Overlapped-step sweep (run via gpurun): bash tools/gpu_ov.sh "ENV=.." ... ; per-side times
set -o pipefail
o=gpurun_out/ov
mkdir -p $o
i=0
for cfg in "$@"; do
  i=$((i+1))
  env JANUS_OVERLAP_TIMING=1 $cfg timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $o/$i.log 2>&1 || { echo "FAIL $cfg"; tail -20 $o/$i.log; exit 1; }
  echo "$cfg : $(grep -o '"ms_per_step": [0-9.]*' $o/$i.log) | $(grep overlap\] $o/$i.log | tail -2 | tr '\n' ' ')"
done
