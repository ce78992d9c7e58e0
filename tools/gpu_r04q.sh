#!/bin/bash
# r04: YIN beside the decode call (JANUS_YIN_BESIDE=<blocks>) vs after it, same box, two
# rounds of 5 timed steps after 2 warm-up; then the driver's default command once
set -o pipefail
out=gpurun_out/r04q
mkdir -p $out
for rep in 1 2; do
for yb in after 128 256; do
  tag=${yb}_$rep
  if [ $yb = after ]; then unset JANUS_YIN_BESIDE; else export JANUS_YIN_BESIDE=$yb; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency --steps 5 --warmup 2 \
    > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'], d['yin_dec_utts'])"
done
done
unset JANUS_YIN_BESIDE
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $out/default.log 2>&1 || { tail -20 $out/default.log; exit 1; }
tail -1 $out/default.log > $out/default.json
python3 -c "
import json; d=json.load(open('$out/default.json')); print('default', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'], d['yin_dec_utts'])"
