#!/bin/bash
# Bench A/B over environment settings (run via gpurun): bash tools/gpu_ab.sh "ENV=.. ENV2=.." "..." ...
# ("-" = defaults). Prints ms/step per setting; logs in gpurun_out/ab/.
set -o pipefail
o=gpurun_out/ab
mkdir -p $o
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=""; [ "$cfg" != "-" ] && envs="$cfg"
  env $envs timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $o/$i.log 2>&1 || { echo "FAIL $cfg"; tail -20 $o/$i.log; exit 1; }
  echo "$cfg : $(grep -o '"ms_per_step": [0-9.]*' $o/$i.log)"
done
