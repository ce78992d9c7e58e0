#!/bin/bash
# r04: fused merge only up to 64 rows (staggered 128-row decoder: merge in the cross-attention
# + block-diagonal value projection): decoder / fallback parity, bench pairs, fallback leg,
# and the driver's torchrun launch form at world size 1
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04m
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_whisper_gpu.py tests/test_pipeline_gpu.py tests/test_bench_config_gpu.py \
  -x -q --timeout 800 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
for cv in 0 1; do
  tag=cvp${cv}_$rep
  if [ $cv = 1 ]; then export JANUS_CVP=1; else unset JANUS_CVP; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['side_ms'], d['roofline']['decoder']['us_per_position'])"
done
done
unset JANUS_CVP
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 1 > $out/fb.log 2>&1 || { tail -20 $out/fb.log; exit 1; }
tail -1 $out/fb.log > $out/fb.json
python3 -c "
import json; d=json.load(open('$out/fb.json')); print('fallback', d['xrt_with_fallback'], d['fallback']['step_ms'])"
bash tools/gpu_torchrun1.sh || exit 1
