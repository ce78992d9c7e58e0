#!/bin/bash
# decoder changes: kernel parity + decode parity tests, then env A/B of the overlapped step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_whisper_gpu.py tests/test_pipeline_gpu.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_pytest.log 2>&1 || { tail -30 gpurun_out/dec_pytest.log; exit 1; }
tail -2 gpurun_out/dec_pytest.log
bash tools/gpu_abenv.sh dec default "JANUS_NO_RESID_LN=1" "JANUS_SKINNY_NO_K1=1" "JANUS_HEAD_ALL_ROUNDS=1" "JANUS_XATTN_CH32=1"
