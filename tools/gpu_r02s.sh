#!/bin/bash
# decoder kernels alone (16 CUs per XCD): default vs LayerNorm-in-prologue
set -o pipefail
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in def lnx; do
  if [ $v = lnx ]; then export JANUS_LN_PROLOGUE=1; else unset JANUS_LN_PROLOGUE; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/ds_$v -o run -- python3 $root/tools/decoder_probe.py --per-xcd 16 --beside 0 --reps 2 > $root/gpurun_out/ds_$v.log 2>&1 || { tail -20 $root/gpurun_out/ds_$v.log; exit 1; }
  grep '{' $root/gpurun_out/ds_$v.log
  f=$(find $root/gpurun_out/ds_$v -name "*.db" | head -1)
  python3 $root/tools/rocprof_stats.py "$f" 14 --csv $root/gpurun_out/ds_$v/kernel_stats.csv | head -16
done
