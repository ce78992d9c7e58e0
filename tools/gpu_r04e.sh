#!/bin/bash
# r04 combined: staggered decoder (tests + same-box bench pairs), the full -m gpu suite,
# shared-encoder groups (bench with xrt_with_fallback), then the vocoder store / staging A/B
set -o pipefail
root=$(pwd)
bash tools/gpu_r04d.sh || exit 1
out=$root/gpurun_out/r04c
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/pytest_all.log 2>&1 || { tail -40 $out/pytest_all.log; exit 1; }
tail -2 $out/pytest_all.log
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
python3 -c "
import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['value'], d['xrt_with_fallback'], d['fallback'])"
bash tools/gpu_store_ab.sh || exit 1
