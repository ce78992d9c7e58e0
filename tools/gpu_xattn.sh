#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k cross_attention > gpurun_out/xt.log 2>&1 || { tail -30 gpurun_out/xt.log; exit 1; }
tail -2 gpurun_out/xt.log
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
JANUS_NO_XABSORB=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_nx.log 2>&1 || { tail -20 gpurun_out/bench_nx.log; exit 1; }
tail -1 gpurun_out/bench_nx.log | cut -c1-300
