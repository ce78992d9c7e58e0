#!/bin/bash
# A/B of experiment builds (JANUS_LIB): tools/gpu_ab.sh tag lib1 lib2 ...  ("default" = in-tree lib)
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = default ]; then unset JANUS_LIB; else export JANUS_LIB=$v; fi
  JANUS_OVERLAP_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --fallback-steps 0 \
    > gpurun_out/ab_${tag}_$v.json 2> gpurun_out/ab_${tag}_$v.err || { tail -5 gpurun_out/ab_${tag}_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/ab_${tag}_$v.json'));print(d['ms_per_step'], d['step_ms'], d['roofline']['avg_launch_ms'])") $(grep overlap gpurun_out/ab_${tag}_$v.err | tail -1)"
done
done
