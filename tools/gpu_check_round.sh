#!/bin/bash
# One GPU call: full -m gpu suite, kernel-trace profile of the timed overlapped steps only
# (--no-idle-latency: no flush, no idle back-to-back steps in the trace), full bench line,
# the BASELINE config 2 / 3 lines and the config-5 stream bench.
# usage (via gpurun): bash tools/gpu_check_round.sh <tag> [skip-tests]  -> gpurun_out/<tag>/
set -o pipefail
tag=${1:-check}
root=$(pwd)
out=$root/gpurun_out/$tag
mkdir -p $out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
  tail -2 $out/pytest.log
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $root/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-idle-latency > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(find $out/prof -name "*.db" | head -1)
python3 $root/tools/rocprof_stats.py "$f" 40 --csv $out/kernel_stats.csv > $out/kernel_top.txt
grep '"metric"' $out/prof.log > $out/bench_under_rocprof.json
cd $root
timeout -k 10 600 python3 -u bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
timeout -k 10 300 python3 -u bench.py --config 2 --steps 5 --warmup 1 > $out/config2.log 2>&1 || { tail -20 $out/config2.log; exit 1; }
tail -1 $out/config2.log > $out/config2.json
timeout -k 10 300 python3 -u bench.py --config 3 --steps 5 --warmup 2 > $out/config3.log 2>&1 || { tail -20 $out/config3.log; exit 1; }
tail -1 $out/config3.log > $out/config3.json
timeout -k 10 300 python3 -u bench.py --config 1 --steps 5 --warmup 1 > $out/config1.log 2>&1 || { tail -20 $out/config1.log; exit 1; }
tail -1 $out/config1.log > $out/config1.json
timeout -k 10 300 python3 -u tools/stream_bench.py --model base.en > $out/stream5.log 2>&1 || { tail -20 $out/stream5.log; exit 1; }
tail -1 $out/stream5.log > $out/stream5.json
python3 $root/tools/conv_avg.py "$(find $out/prof -name "*.db" | head -1)" $out/bench_under_rocprof.json > $out/conv_avg.txt || true
cut -c1-900 $out/bench.json
cat $out/conv_avg.txt
head -12 $out/kernel_top.txt
