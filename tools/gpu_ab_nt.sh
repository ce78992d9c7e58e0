#!/bin/bash
# A/B: default vs non-temporal vocoder activation traffic variants (JANUS_LIB)
set -o pipefail
mkdir -p gpurun_out
for v in default nt nst default nt nst; do
  case $v in nt) export JANUS_LIB=libjanus_hip_nt.so;; nst) export JANUS_LIB=libjanus_hip_nst.so;; *) unset JANUS_LIB;; esac
  JANUS_OVERLAP_TIMING=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/ab_nt_$v.json 2> gpurun_out/ab_nt_$v.err || exit $?
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/ab_nt_$v.json'));print(d['ms_per_step'], d['step_ms'], d['roofline']['avg_launch_ms'])") $(grep overlap gpurun_out/ab_nt_$v.err | tail -1)"
done
