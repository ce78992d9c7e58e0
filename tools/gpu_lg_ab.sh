#!/bin/bash
# vocabulary-projection kernel duration under build / env variants (decoder alone, 16 CUs
# per XCD, 64 positions): bash tools/gpu_lg_ab.sh "ENV=.." ...   (X=1 = default)
set -o pipefail
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  tag=$(echo $v | tr '=' '_' | tr -d ' ')
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/lg_$tag -o run --output-format csv -- python3 $root/tools/decoder_probe.py --per-xcd 16 --beside 0 --reps 2 --max-length 64 > $root/gpurun_out/lg_$tag.log 2>&1 || { tail -5 $root/gpurun_out/lg_$tag.log; exit 1; }
  f=$(find $root/gpurun_out/lg_$tag -name "*kernel_stats.csv" | head -1)
  echo "$v: $(grep -E 'logits_partial|select_partials' $f | cut -d, -f1-5 | tr '\n' ' ' | cut -c1-300)"
done
