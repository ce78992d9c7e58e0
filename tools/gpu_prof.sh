#!/bin/bash
# Kernel-trace profile of a short bench run (run via gpurun). $1 = tag
set -o pipefail
tag=${1:-prof}
mkdir -p gpurun_out
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/$tag -o run -- python3 $root/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $root/gpurun_out/$tag.log 2>&1 || { tail -20 $root/gpurun_out/$tag.log; exit 1; }
grep '"metric"' $root/gpurun_out/$tag.log | cut -c1-400
f=$(find $root/gpurun_out/$tag -name "*.db" | head -1)
python3 $root/tools/rocprof_stats.py "$f" 40 --csv $root/gpurun_out/$tag/kernel_stats.csv
