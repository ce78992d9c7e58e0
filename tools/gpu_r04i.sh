#!/bin/bash
# r04: staggered step as the bench default — parity (incl. the bench-size rows through the
# staggered step), YIN split fine sweep, vocoder store / staging A/B in the new regime
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04i
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests/test_pipeline_gpu.py tests/test_bench_config_gpu.py -x -v --timeout 900 \
  --timeout-method thread -k "stagger or pipelined or bench_workload" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for yd in 36 40 44 48; do
  JANUS_YIN_DEC_UTTS=$yd timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency \
    > $out/yd$yd.log 2>&1 || { tail -20 $out/yd$yd.log; exit 1; }
  tail -1 $out/yd$yd.log > $out/yd$yd.json
  python3 -c "
import json; d=json.load(open('$out/yd$yd.json')); print('yd$yd', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'])"
done
for xs in 2 8 4; do
  JANUS_XATTN_SPLITS=$xs timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency \
    > $out/xs$xs.log 2>&1 || { tail -20 $out/xs$xs.log; exit 1; }
  tail -1 $out/xs$xs.log > $out/xs$xs.json
  python3 -c "
import json; d=json.load(open('$out/xs$xs.json')); print('xsplit$xs', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'])"
done
bash tools/gpu_ab.sh store default libjanus_hip_stplain.so libjanus_hip_wt.so libjanus_hip_stwt.so || exit 1
