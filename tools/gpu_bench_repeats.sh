#!/bin/bash
# three default bench lines back to back on one box (box-to-box and run-to-run spread)
set -o pipefail
out=gpurun_out/bench_repeats
mkdir -p $out
for r in 1 2 3; do
  timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $out/b$r.log 2>&1 || { tail -20 $out/b$r.log; exit 1; }
  tail -1 $out/b$r.log > $out/b$r.json
  python3 -c "
import json; d=json.load(open('$out/b$r.json')); print($r, d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'], d['yin_dec_utts'], d['xrt_with_fallback'])"
done
for yb in ${YB:-}; do
  JANUS_YIN_BESIDE=$yb timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency \
    --steps 5 --warmup 2 > $out/yb$yb.log 2>&1 || { tail -20 $out/yb$yb.log; exit 1; }
  tail -1 $out/yb$yb.log > $out/yb$yb.json
  python3 -c "
import json; d=json.load(open('$out/yb$yb.json')); print('beside$yb', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'], d['yin_dec_utts'])"
done
