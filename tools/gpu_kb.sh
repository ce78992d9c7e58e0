#!/bin/bash
# kernel tests + conv/unit microbench (run via gpurun)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_vocoder_gpu.py -x -q > gpurun_out/kt.log 2>&1 || { tail -30 gpurun_out/kt.log; exit 1; }
tail -2 gpurun_out/kt.log
timeout -k 10 200 python tools/kbench.py > gpurun_out/kb.log 2>&1 || { tail -20 gpurun_out/kb.log; exit 1; }
grep -v amdgpu.ids gpurun_out/kb.log
