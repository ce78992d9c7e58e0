#!/bin/bash
# bench A/B over env settings / builds: tools/gpu_ab_env.sh tag default env:A=1,B=2 lib:libx.so ...
# (env: comma-separated NAME=VALUE pairs applied to the in-tree lib)
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
reps=${AB_REPS:-2}
for rep in $(seq $reps); do
for v in "$@"; do
  unset JANUS_LIB
  envs=""
  case "$v" in
    default) ;;
    env:*) envs="${v#env:}"; envs="${envs//,/ }" ;;
    lib:*) export JANUS_LIB="${v#lib:}" ;;
  esac
  name=$(echo "$v" | tr -c 'A-Za-z0-9_=.\n' '_')
  env $envs JANUS_OVERLAP_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/ab_${tag}_$name.json 2> gpurun_out/ab_${tag}_$name.err || { tail -5 gpurun_out/ab_${tag}_$name.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/ab_${tag}_$name.json'));print(d['ms_per_step'], d['step_ms'], d['roofline']['avg_launch_ms'])") $(grep overlap gpurun_out/ab_${tag}_$name.err | tail -1)"
done
done
