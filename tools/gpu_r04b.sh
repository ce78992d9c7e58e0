#!/bin/bash
# r04: shared-encoder fallback decode (tests + bench line with xrt_with_fallback), then the
# staging-policy A/B round 2
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04b
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py tests/test_pipeline_gpu.py -x -v --timeout 300 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
python3 -c "
import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['value'], d['xrt_with_fallback'], d['fallback'])"
bash tools/gpu_halo_ab2.sh || exit 1
