#!/bin/bash
# Round deliverables on one box: conv HBM traffic (PMC), kernel-trace profile, full bench line.
# usage (via gpurun): bash tools/gpu_final.sh <tag>   -> gpurun_out/final_<tag>/
set -o pipefail
tag=${1:-r01}
root=$(pwd)
out=$root/gpurun_out/final_$tag
mkdir -p $out
bash tools/gpu_traffic.sh > $out/traffic.log 2>&1 || { tail -5 $out/traffic.log; exit 1; }
cp $root/gpurun_out/traffic/traffic.json $root/profiles/traffic_r01.json
cp $root/gpurun_out/traffic/traffic.json $out/traffic_r01.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $root/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(find $out/prof -name "*.db" | head -1)
python3 $root/tools/rocprof_stats.py "$f" 25 --csv $out/kernel_stats.csv > $out/kernel_top.txt
cd $root
timeout -k 10 600 python3 bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
cat $out/bench.json
head -12 $out/kernel_top.txt
