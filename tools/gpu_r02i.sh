#!/bin/bash
set -o pipefail
bash tools/gpu_traffic.sh || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/traffic/traffic.json'))
print('total x', round(d['traffic_over_algorithmic'],3))
for k,v in d['by_family'].items(): print(k, v['launches'], round(v['traffic_over_algorithmic'],3))
"
bash tools/gpu_abenv.sh remap default "JANUS_CONV_REMAP=3" "JANUS_LIB=libjanus_hip_nr.so JANUS_CONV_REMAP=0"
