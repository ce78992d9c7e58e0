#!/bin/bash
# r05: host tail prefetched behind the decoder call: pipeline parity, then step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_pipeline_gpu.py::test_staggered_step_matches_sequential" > gpurun_out/r05g_tests.log 2>&1 || { tail -30 gpurun_out/r05g_tests.log; exit 1; }
tail -2 gpurun_out/r05g_tests.log
AB_REPS=2 bash tools/gpu_ab_env.sh hostpf default env:JANUS_HOST_PREFETCH=0 env:JANUS_VOC_WAIT_ENC=0 env:JANUS_VOC_WAIT_ENC=0,JANUS_VOC_DEC_UTTS=1
