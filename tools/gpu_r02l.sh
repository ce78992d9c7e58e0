#!/bin/bash
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/l_test.log 2>&1 || { tail -30 gpurun_out/l_test.log; exit 1; }
tail -1 gpurun_out/l_test.log
bash tools/gpu_abenv.sh xd default "JANUS_XATTN_DEPTH=1" "JANUS_XATTN_DEPTH=3"
