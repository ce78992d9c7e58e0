#!/bin/bash
# r04 staging cache policy, round 2: halo rows kept (default) vs every C = 64 / 32 staged
# row kept (libjanus_hip_stplain.so) vs r03's all non-temporal (libjanus_hip_halont.so)
set -o pipefail
root=$(pwd)
mkdir -p gpurun_out
JANUS_LIB=libjanus_hip_stplain.so bash tools/gpu_traffic.sh traffic_stplain || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/traffic_stplain/traffic.json'))
print('stplain', round(d['traffic_over_algorithmic'],3), {k: round(v['traffic_over_algorithmic'],3) for k,v in d['by_family'].items()})
"
bash tools/gpu_ab.sh halo2 default libjanus_hip_stplain.so libjanus_hip_halont.so || exit 1
