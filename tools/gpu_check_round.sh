#!/bin/bash
# One GPU call: full -m gpu suite, kernel-trace profile of a short bench, full bench line.
# usage (via gpurun): bash tools/gpu_check_round.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
tag=${1:-check}
root=$(pwd)
out=$root/gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $root/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(find $out/prof -name "*.db" | head -1)
python3 $root/tools/rocprof_stats.py "$f" 40 --csv $out/kernel_stats.csv > $out/kernel_top.txt
grep '"metric"' $out/prof.log > $out/bench_under_rocprof.json
cd $root
timeout -k 10 600 python3 -u bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
cat $out/bench.json | cut -c1-600
head -12 $out/kernel_top.txt
