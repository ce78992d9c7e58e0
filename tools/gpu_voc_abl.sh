#!/bin/bash
# standalone vocoder timing per family for A/B or ablation builds (no tests: ablation
# builds compute wrong results on purpose)
# usage: bash tools/gpu_voc_abl.sh default libjanus_hip_x.so env:NAME=VALUE ...
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in "$@"; do
  unset JANUS_LIB
  case "$v" in
    default) envs="" ;;
    env:*) envs="${v#env:}"; envs="${envs//,/ }" ;;
    *) export JANUS_LIB=$v; envs="" ;;
  esac
  env $envs timeout -k 10 200 python -u tools/vocoder_ab.py --reps 3 2> gpurun_out/voc_ab.err | tail -1 || { tail -5 gpurun_out/voc_ab.err; exit 1; }
done
done
