#!/bin/bash
# r04 halo cache policy: vocoder tests, same-box bench A/B (default = halo rows default policy,
# libjanus_hip_halont.so = every staging load non-temporal, r03) and PMC traffic of both
set -o pipefail
root=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vocoder_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/halo_pytest.log 2>&1 || { tail -30 gpurun_out/halo_pytest.log; exit 1; }
tail -1 gpurun_out/halo_pytest.log
bash tools/gpu_ab.sh halo default libjanus_hip_halont.so || exit 1
bash tools/gpu_traffic.sh traffic_halo || exit 1
JANUS_LIB=libjanus_hip_halont.so bash tools/gpu_traffic.sh traffic_halont || exit 1
python3 -c "
import json
for t in ('traffic_halo','traffic_halont'):
    d=json.load(open('gpurun_out/%s/traffic.json'%t))
    print(t, round(d['traffic_over_algorithmic'],3), {k: round(v['traffic_over_algorithmic'],3) for k,v in d['by_family'].items()})
"
