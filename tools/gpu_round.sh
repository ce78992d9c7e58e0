#!/bin/bash
# tests, microbench, conv traffic, bench (run via gpurun)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 200 python tools/kbench.py > gpurun_out/kb.log 2>&1 || { tail -20 gpurun_out/kb.log; exit 1; }
grep -v amdgpu.ids gpurun_out/kb.log
bash tools/gpu_traffic.sh || exit 1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
