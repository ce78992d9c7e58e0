#!/bin/bash
# r04: shared-encoder GROUP cross-attention (tests + bench with xrt_with_fallback), then the
# store / staging policy A/B
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04c
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py -x -v --timeout 300 \
  --timeout-method thread -k "shared or seek_loop or sample" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
python3 -c "
import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['value'], d['xrt_with_fallback'], d['fallback'])"
bash tools/gpu_store_ab.sh || exit 1
# decoder cost at 128 rows per decode (two batches' worth) on the overlapped step's partition
timeout -k 10 600 python3 -u bench.py --batch 128 --steps 2 --warmup 1 --no-cpu-baseline --fallback-steps 0 \
  --no-idle-latency > $out/bench_b128.log 2>&1 || { tail -20 $out/bench_b128.log; exit 1; }
tail -1 $out/bench_b128.log > $out/bench_b128.json
python3 -c "
import json; d=json.load(open('$out/bench_b128.json')); print('B=128', d['ms_per_step'], d['side_ms'], d['roofline']['decoder']['us_per_position'])"
