#!/bin/bash
# r02: vocoder PMC traffic (per family) + kernel-trace profile of the bench
set -o pipefail
bash tools/gpu_traffic.sh || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/traffic/traffic.json'))
print('total x', round(d['traffic_over_algorithmic'],3))
for k,v in d['by_family'].items(): print(k, v['launches'], round(v['traffic_over_algorithmic'],3), round(v['fetch_bytes']/1e9,1), round(v['write_bytes']/1e9,1), round(v['algorithmic_bytes']/1e9,1))
"
bash tools/gpu_prof.sh r02_v2 || exit 1
head -30 gpurun_out/r02_v2/kernel_stats.csv
