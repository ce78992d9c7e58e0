#!/bin/bash
# vocoder parity tests, then standalone vocoder timing per family for each lib (A/B builds)
# usage: bash tools/gpu_voc_ab.sh default libjanus_hip_x.so ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_vocoder_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/voc_pytest.log 2>&1 || { tail -30 gpurun_out/voc_pytest.log; exit 1; }
tail -1 gpurun_out/voc_pytest.log
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = default ]; then unset JANUS_LIB; else export JANUS_LIB=$v; fi
  timeout -k 10 200 python -u tools/vocoder_ab.py --reps 3 2> gpurun_out/voc_ab.err | tail -1 || { tail -5 gpurun_out/voc_ab.err; exit 1; }
done
done
