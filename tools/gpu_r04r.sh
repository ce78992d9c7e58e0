#!/bin/bash
# r04: YIN-beside grid cap fine sweep (same box, 5 timed steps after 2 warm-up, two rounds)
set -o pipefail
out=gpurun_out/r04r
mkdir -p $out
for rep in 1 2; do
for yb in 128 96 192; do
  tag=yb${yb}_$rep
  JANUS_YIN_BESIDE=$yb timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency \
    --steps 5 --warmup 2 > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['side_ms'], d['yin_dec_utts'])"
done
done
