#!/bin/bash
# r04: N slot sets in the staggered decoder (JANUS_STAGGER_SETS): parity for 2 / 3 / 4,
# then same-box bench points (self-balancing YIN split)
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04p
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_whisper_gpu.py -x -q --timeout 300 \
  --timeout-method thread -k "stagger" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for cfg in ${CFGS:-"2,2" "3,2" "4,2" "4,1" "2,2"}; do
  set -- ${cfg//,/ }
  tag=sets$1_xs$2
  JANUS_STAGGER_SETS=$1 JANUS_XATTN_SPLITS=$2 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 \
    --no-idle-latency --steps 5 --warmup 2 > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['side_ms'], d['yin_dec_utts'], d['roofline']['decoder']['us_per_position'], d['p50_latency_ms'])"
done
