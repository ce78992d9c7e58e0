#!/bin/bash
# per-row-block fused LayerNorm (JANUS_LN_FUSE): decode parity under it, then the step A/B
set -o pipefail
mkdir -p gpurun_out
JANUS_LN_FUSE=1 timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py tests/test_pipeline_gpu.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/lnf_pytest.log 2>&1 || { tail -30 gpurun_out/lnf_pytest.log; exit 1; }
tail -1 gpurun_out/lnf_pytest.log
bash tools/gpu_abenv.sh lnf default "JANUS_LN_FUSE=1"
