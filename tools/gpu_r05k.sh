#!/bin/bash
# r05: C = 64 units compiled per (k, d): vocoder parity, standalone forward A/B, step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vocoder_gpu.py \
  -k "generator_rms or family_stats" > gpurun_out/r05k_tests.log 2>&1 || { tail -30 gpurun_out/r05k_tests.log; exit 1; }
tail -2 gpurun_out/r05k_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "resunit or wide" > gpurun_out/r05k_tests2.log 2>&1 || { tail -30 gpurun_out/r05k_tests2.log; exit 1; }
tail -2 gpurun_out/r05k_tests2.log
for r in 1 2; do
  timeout -k 10 200 python3 tools/vocoder_ab.py --reps 3 || exit 1
  JANUS_WIDE_LDS_RT=1 timeout -k 10 200 python3 tools/vocoder_ab.py --reps 3 || exit 1
done
AB_REPS=2 bash tools/gpu_ab_env.sh c64kd default env:JANUS_WIDE_LDS_RT=1
