#!/bin/bash
# r05: the layer kernel (persistent = 2): parity tests, stamps, step A/B against persistent = 1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_whisper_gpu.py::test_persistent_segments_vs_oracle" \
  "tests/test_whisper_gpu.py::test_persistent_staggered_bit_identical" > gpurun_out/r05l_tests.log 2>&1 || { tail -40 gpurun_out/r05i_tests.log; exit 1; }
tail -2 gpurun_out/r05l_tests.log
JANUS_DEC_PERSIST=2 JANUS_LIB=libjanus_hip_prof.so JANUS_SEG_PROF=2 timeout -k 10 300 python3 tools/seg_prof.py > gpurun_out/segprof7.txt 2>&1 || { tail -5 gpurun_out/segprof5.txt; exit 1; }
tail -1 gpurun_out/segprof7.txt | cut -c1-600
AB_REPS=3 bash tools/gpu_ab_env.sh layerk4 default env:JANUS_DEC_PERSIST=2
