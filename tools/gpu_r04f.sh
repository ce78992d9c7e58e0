#!/bin/bash
# r04: staggered decoder (tests + same-box bench pairs), the encoder GEMM schedule A/B, the
# default bench line (xrt_with_fallback), then the full -m gpu suite in the time that is left
set -o pipefail
root=$(pwd)
bash tools/gpu_r04d.sh || exit 1
bash tools/gpu_gemm_pp.sh || exit 1
out=$root/gpurun_out/r04f
mkdir -p $out
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
python3 -c "
import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['value'], d['xrt_with_fallback'], d['fallback'])"
left=$((1140 - SECONDS))
echo "pytest budget ${left}s"
[ $left -gt 120 ] || exit 0
timeout -k 10 $left python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/pytest_all.log 2>&1 || { tail -40 $out/pytest_all.log; exit 1; }
tail -2 $out/pytest_all.log
