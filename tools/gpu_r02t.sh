#!/bin/bash
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_test.log 2>&1 || { tail -40 gpurun_out/t_test.log; exit 1; }
tail -1 gpurun_out/t_test.log
bash tools/gpu_abenv.sh lnm default JANUS_LN_PROLOGUE=0 JANUS_LN_PROLOGUE=9 JANUS_LN_PROLOGUE=5
