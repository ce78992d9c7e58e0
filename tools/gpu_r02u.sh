#!/bin/bash
# full GPU suite + final bench line + kernel-trace profile (r02 v3)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/u_test.log 2>&1 || { tail -40 gpurun_out/u_test.log; exit 1; }
tail -2 gpurun_out/u_test.log
timeout -k 10 600 python -u bench.py > gpurun_out/u_bench.json 2> gpurun_out/u_bench.err || { tail -20 gpurun_out/u_bench.err; exit 1; }
cut -c1-300 gpurun_out/u_bench.json
bash tools/gpu_prof.sh r02_v3
