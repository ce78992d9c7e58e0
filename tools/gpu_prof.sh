#!/bin/bash
# kernel-trace profile of the timed staggered steps only (--no-idle-latency) -> gpurun_out/<tag>/
set -o pipefail
tag=${1:-prof}
root=$(pwd)
out=$root/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $root/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-idle-latency > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(find $out/prof -name "*.db" | head -1)
python3 $root/tools/rocprof_stats.py "$f" 60 --csv $out/kernel_stats.csv > $out/kernel_top.txt
grep '"metric"' $out/prof.log > $out/bench_under_rocprof.json
cd $root
python3 tools/conv_avg.py "$f" $out/bench_under_rocprof.json > $out/conv_avg.txt || true
head -40 $out/kernel_top.txt | cut -c1-150
