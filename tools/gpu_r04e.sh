#!/bin/bash
# r04 combined: staggered decoder (tests + same-box bench pairs), shared-encoder groups (tests +
# bench with xrt_with_fallback), then the vocoder store / staging policy A/B
set -o pipefail
root=$(pwd)
bash tools/gpu_r04d.sh || exit 1
out=$root/gpurun_out/r04c
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py -x -v --timeout 300 \
  --timeout-method thread -k "seek_loop or sample" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
python3 -c "
import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['value'], d['xrt_with_fallback'], d['fallback'])"
bash tools/gpu_store_ab.sh || exit 1
