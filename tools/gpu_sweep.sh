#!/bin/bash
# GPU tuning pass: gpu tests, fused-unit tile sweep, short bench (run via gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
for bm in 0 256 64; do
  JANUS_RU_BM=$bm timeout -k 10 120 python tools/kbench.py --units-only > gpurun_out/units_bm$bm.log 2>&1 || exit 1
  echo "BM=$bm"; cat gpurun_out/units_bm$bm.log
done
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
