#!/bin/bash
# r05: persistent-segment L2 touch + load order: parity tests, phase stamps, bench A/B vs the previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_whisper_gpu.py::test_persistent_segments_vs_oracle" \
  "tests/test_whisper_gpu.py::test_persistent_staggered_bit_identical" \
  "tests/test_pipeline_gpu.py::test_staggered_step_matches_sequential" > gpurun_out/r05h_tests.log 2>&1 || { tail -30 gpurun_out/r05f_tests.log; exit 1; }
tail -2 gpurun_out/r05h_tests.log
JANUS_LIB=libjanus_hip_prof.so JANUS_SEG_PROF=2 timeout -k 10 300 python3 tools/seg_prof.py > gpurun_out/segprof4.txt 2>&1 || { tail -5 gpurun_out/segprof3.txt; exit 1; }
tail -1 gpurun_out/segprof4.txt
AB_REPS=2 bash tools/gpu_ab_env.sh r05h default lib:libjanus_hip_old.so
