#!/bin/bash
# Round deliverables in one GPU call: full -m gpu suite, free-running decode parity
# (base.en 8 / tiny.en 16 utterances, decoder-only and end to end), kernel-trace profile of
# a short bench, full bench line (with the measured CPU baseline).
# usage (via gpurun): bash tools/gpu_round_final.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
tag=${1:-final}
root=$(pwd)
out=$root/gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -u tools/decode_parity.py --model base.en --n 8 --e2e > $out/parity_base.json 2> $out/parity_base.err || { tail -5 $out/parity_base.err; exit 1; }
timeout -k 10 400 python -u tools/decode_parity.py --model tiny.en --n 16 --e2e > $out/parity_tiny.json 2> $out/parity_tiny.err || { tail -5 $out/parity_tiny.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $root/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
f=$(find $out/prof -name "*.db" | head -1)
python3 $root/tools/rocprof_stats.py "$f" 40 --csv $out/kernel_stats.csv > $out/kernel_top.txt
cd $root
JANUS_OVERLAP_TIMING=1 timeout -k 10 600 python3 -u bench.py > $out/bench.log 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -1 $out/bench.log > $out/bench.json
grep overlap $out/bench.err | tail -3
cut -c1-300 $out/bench.json
