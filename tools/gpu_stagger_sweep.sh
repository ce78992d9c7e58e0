#!/bin/bash
# r04: staggered step, YIN split sweep (utterances whose YIN runs on the decoder side)
set -o pipefail
out=gpurun_out/stag_sweep
mkdir -p $out
for yd in 0 16 32 48; do
  JANUS_YIN_DEC_UTTS=$yd timeout -k 10 300 python3 -u bench.py --stagger 1 --steps 3 --warmup 1 --no-cpu-baseline \
    --fallback-steps 0 --no-idle-latency > $out/yd$yd.log 2>&1 || { tail -20 $out/yd$yd.log; exit 1; }
  tail -1 $out/yd$yd.log > $out/yd$yd.json
  python3 -c "
import json; d=json.load(open('$out/yd$yd.json')); print('yin_dec $yd', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'])"
done
