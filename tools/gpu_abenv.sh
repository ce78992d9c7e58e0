#!/bin/bash
# A/B of runtime variants: tools/gpu_abenv.sh tag "ENV=.. ENV2=.." "..." ("default" = no env)
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
i=0
for rep in 1 2; do
for v in "$@"; do
  i=$((i+1))
  if [ "$v" = default ]; then envs=""; else envs="$v"; fi
  env $envs JANUS_OVERLAP_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/abe_${tag}_$i.json 2> gpurun_out/abe_${tag}_$i.err || { tail -5 gpurun_out/abe_${tag}_$i.err; exit 1; }
  echo "[$v] $(python -c "
import json;d=json.load(open('gpurun_out/abe_${tag}_$i.json'))
print(d['ms_per_step'], d['step_ms'], [(f['family'], round(f['ms']/f['launches']*(6 if f['family']=='conv' else 9),2)) for f in d['roofline']['families']])") $(grep overlap gpurun_out/abe_${tag}_$i.err | tail -1)"
done
done
