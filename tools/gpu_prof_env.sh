#!/bin/bash
# Kernel-trace profile of a short bench run under extra environment (run via gpurun).
# usage: bash tools/gpu_prof_env.sh <tag> [ENV=VAL ...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
root=$(pwd)
for kv in "$@"; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/$tag -o run -- python3 $root/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $root/gpurun_out/$tag.log 2>&1 || { tail -20 $root/gpurun_out/$tag.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $root/gpurun_out/$tag.log
f=$(find $root/gpurun_out/$tag -name "*.db" | head -1)
python3 $root/tools/rocprof_stats.py "$f" 30 --csv $root/gpurun_out/$tag/kernel_stats.csv
