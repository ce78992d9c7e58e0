#!/bin/bash
# r04: encoder GEMM schedules — gemm_big double-buffered (default) vs ping-pong
# (JANUS_GEMM_BIG=pp): bit-identity tests, then interleaved timing rounds in one process
set -o pipefail
out=gpurun_out/gemm_pp
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_big" -x -q --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
GEMM_FNS=janus_gemm_f16,janus_gemm_nt128_f16 GEMM_VARIANTS=dbuf,pp GEMM_ROUNDS=7 timeout -k 10 300 \
  python3 -u tools/gemm_big_probe.py > $out/probe.jsonl 2>&1 || { tail -20 $out/probe.jsonl; exit 1; }
cat $out/probe.jsonl
