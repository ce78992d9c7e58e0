#!/bin/bash
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py tests/test_pipeline_gpu.py tests/test_vocoder_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/o_test.log 2>&1 || { tail -30 gpurun_out/o_test.log; exit 1; }
tail -1 gpurun_out/o_test.log
bash tools/gpu_abenv.sh lg default "JANUS_LG_DEPTH=2" "JANUS_LN_PROLOGUE=1" "JANUS_FUSED_LN=1" "JANUS_XATTN_SPLITS=3" || exit 1
bash tools/gpu_r02m.sh
