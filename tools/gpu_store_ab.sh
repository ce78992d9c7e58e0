#!/bin/bash
# r04: vocoder store / staging cache policy A/B on one box (overlapped bench step):
# default (halo rows kept, nt stores), stplain (C = 64 / 32 staging kept), wt (write-through
# sc1 stores), stwt (both); vocoder parity under the write-through build first
set -o pipefail
mkdir -p gpurun_out
JANUS_LIB=libjanus_hip_stwt.so timeout -k 10 300 python -u -m pytest tests/test_vocoder_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/stwt_pytest.log 2>&1 || { tail -30 gpurun_out/stwt_pytest.log; exit 1; }
tail -1 gpurun_out/stwt_pytest.log
bash tools/gpu_ab.sh store default libjanus_hip_stplain.so libjanus_hip_wt.so libjanus_hip_stwt.so || exit 1
