#!/bin/bash
# r04: self-balancing YIN split (default) vs the fixed 40 of 64: parity, then same-box pairs
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04n
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "stagger" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
for mode in auto 40; do
  tag=${mode}_$rep
  if [ $mode = auto ]; then unset JANUS_YIN_DEC_UTTS; else export JANUS_YIN_DEC_UTTS=$mode; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency --steps 5 --warmup 2 \
    > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'], d['yin_dec_utts'])"
done
done
