#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_vocoder_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "resunit or generator or family or conv" > gpurun_out/p_test.log 2>&1 || { tail -30 gpurun_out/p_test.log; exit 1; }
tail -1 gpurun_out/p_test.log
bash tools/gpu_abenv.sh epi default JANUS_LIB=libjanus_hip_old.so || exit 1
bash tools/gpu_pmc_voc.sh
