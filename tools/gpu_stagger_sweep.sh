#!/bin/bash
# r04: staggered step, sweep of the decoder's CUs per XCD (--overlap) and of the YIN split
# (utterances whose YIN runs on the decoder side)
set -o pipefail
out=gpurun_out/stag_sweep
mkdir -p $out
for cfg in "16 16" "16 32" "14 0" "14 16" "12 0"; do
  set -- $cfg
  ov=$1; yd=$2; tag=ov${ov}_yd${yd}
  JANUS_YIN_DEC_UTTS=$yd timeout -k 10 300 python3 -u bench.py --stagger 1 --overlap $ov --steps 3 --warmup 1 \
    --no-cpu-baseline --fallback-steps 0 --no-idle-latency > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'])"
done
