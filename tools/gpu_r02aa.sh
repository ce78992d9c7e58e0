#!/bin/bash
# logits kernel duration under variations (decoder alone, 16 CUs per XCD, 64 positions)
set -o pipefail
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in "X=1" "JANUS_LOGITS_BLOCKS=256" "JANUS_LOGITS_BLOCKS=64" "JANUS_LN_PROLOGUE=1" "JANUS_LG_DEPTH=2"; do
  tag=$(echo $v | tr '=' '_')
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/lg_$tag -o run --output-format csv -- python3 $root/tools/decoder_probe.py --per-xcd 16 --beside 0 --reps 2 --max-length 64 > $root/gpurun_out/lg_$tag.log 2>&1 || { tail -5 $root/gpurun_out/lg_$tag.log; exit 1; }
  f=$(find $root/gpurun_out/lg_$tag -name "*kernel_stats.csv" | head -1)
  echo "$v: $(grep -E 'logits_partial|layernorm' $f | cut -d, -f1-5 | tr '\n' ' ' | cut -c1-300)"
done
