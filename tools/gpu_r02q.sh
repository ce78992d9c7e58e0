#!/bin/bash
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py tests/test_pipeline_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/q_test.log 2>&1 || { tail -40 gpurun_out/q_test.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/q_test.log | tail -25
bash tools/gpu_abenv.sh lt default JANUS_ENC_BLASLT=0
