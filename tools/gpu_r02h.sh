#!/bin/bash
# r02: XCD-aware vocoder tile order — parity, traffic per family, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_vocoder_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/h_test.log 2>&1 || { tail -30 gpurun_out/h_test.log; exit 1; }
tail -2 gpurun_out/h_test.log
bash tools/gpu_traffic.sh || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/traffic/traffic.json'))
print('total x', round(d['traffic_over_algorithmic'],3))
for k,v in d['by_family'].items(): print(k, v['launches'], round(v['traffic_over_algorithmic'],3), round(v['fetch_bytes']/1e9,1), round(v['write_bytes']/1e9,1), round(v['algorithmic_bytes']/1e9,1))
"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/h_bench.log 2>&1 || { tail -20 gpurun_out/h_bench.log; exit 1; }
grep '"metric"' gpurun_out/h_bench.log | cut -c1-600
