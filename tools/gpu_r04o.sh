#!/bin/bash
# r04: LayerNorm launches above 64 rows: decoder parity (shared rows > 64, staggered, bench
# rows), same-box bench pairs against the prologue mask 9, fallback leg
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04o
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_whisper_gpu.py tests/test_pipeline_gpu.py tests/test_bench_config_gpu.py \
  -x -q --timeout 800 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
for m in auto 9; do
  tag=ln${m}_$rep
  if [ $m = auto ]; then unset JANUS_LN_PROLOGUE; else export JANUS_LN_PROLOGUE=$m; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency --steps 5 --warmup 2 \
    > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'], d['yin_dec_utts'], d['roofline']['decoder']['us_per_position'])"
done
done
unset JANUS_LN_PROLOGUE
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 1 > $out/fb.log 2>&1 || { tail -20 $out/fb.log; exit 1; }
tail -1 $out/fb.log > $out/fb.json
python3 -c "
import json; d=json.load(open('$out/fb.json')); print('fallback', d['xrt_with_fallback'], d['fallback']['step_ms'])"
