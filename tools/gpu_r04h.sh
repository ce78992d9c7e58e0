#!/bin/bash
# r04: three-lane step with the vocoder / encoder lanes enqueued ahead of the decoder call:
# parity, then lane splits against the best staggered point (same box)
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04h
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_whisper_gpu.py tests/test_kernels_gpu.py \
  -x -v --timeout 200 --timeout-method thread -k "${TESTK:-pipelined or shared_encoder or gemm_big}" \
  > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
# configs: stagger,overlap,enc_cus,yin_dec_utts
CFGS=${CFGS:-"1,16,0,32 2,16,0,0 2,16,0,16 1,16,0,24 1,16,0,40 2,16,0,8 1,16,0,32"}
for cfg in $CFGS; do
  set -- ${cfg//,/ }
  tag=s$1_ov$2_e$3_yd$4
  JANUS_YIN_DEC_UTTS=$4 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency \
    --stagger $1 --overlap $2 --enc-cus $3 > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'])"
done
