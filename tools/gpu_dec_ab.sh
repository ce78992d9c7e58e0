#!/bin/bash
# decoder changes: kernel parity + decode parity tests, then env A/B of the overlapped step
# usage: bash tools/gpu_dec_ab.sh tag "ENV=.." ...   (default always first)
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_whisper_gpu.py tests/test_pipeline_gpu.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_pytest.log 2>&1 || { tail -30 gpurun_out/dec_pytest.log; exit 1; }
tail -1 gpurun_out/dec_pytest.log
bash tools/gpu_abenv.sh $tag default "$@"
