#!/bin/bash
# r04: three-lane step (encoder on its own CU lane) parity + lane-split bench points,
# staggered-step CU / YIN sweep, fallback cross-attention groups vs pairs (same box),
# encoder GEMM schedules (dbuf / k-rotated / ping-pong) in one process
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04g
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "pipelined or staggered_step" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for cfg in "1 16 0" "2 16 4" "2 16 2" "2 20 4" "2 18 2"; do
  set -- $cfg
  tag=s$1_ov$2_e$3
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency --stagger $1 \
    --overlap $2 --enc-cus $3 > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'])"
done
bash tools/gpu_stagger_sweep.sh || exit 1
for rep in 1 2; do
for ng in 0 1; do
  if [ $ng = 1 ]; then export JANUS_NO_XGROUP=1; else unset JANUS_NO_XGROUP; fi
  timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 1 \
    > $out/fb_ng${ng}_$rep.log 2>&1 || { tail -20 $out/fb_ng${ng}_$rep.log; exit 1; }
  tail -1 $out/fb_ng${ng}_$rep.log > $out/fb_ng${ng}_$rep.json
  python3 -c "
import json; d=json.load(open('$out/fb_ng${ng}_$rep.json')); print('no_xgroup $ng', d['ms_per_step'], d['xrt_with_fallback'], d['fallback']['step_ms'])"
done
done
unset JANUS_NO_XGROUP
GEMM_FNS=janus_gemm_f16 GEMM_VARIANTS=dbuf,rot,pp GEMM_ROUNDS=7 timeout -k 10 300 \
  python3 -u tools/gemm_big_probe.py > $out/probe.jsonl 2>&1 || { tail -20 $out/probe.jsonl; exit 1; }
cat $out/probe.jsonl
