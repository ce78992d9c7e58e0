#!/bin/bash
# bench A/B over env settings / builds, timed steps only (--no-idle-latency):
#   tools/gpu_ab_env.sh tag default env:A=1,B=2 lib:libx.so lib:libx.so+env:A=1 ...
# (env: comma-separated NAME=VALUE pairs: ServingTuning fields, or kernel switches with a
# -DJANUS_AB_KNOBS lib; lib: an alternative in-tree build, JANUS_LIB)
# AB_REPS rounds (default 2), AB_STEPS timed steps (default 5). One line per run:
# variant, ms/step, mean vocoder / decoder side, conv avg launch ms.
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
reps=${AB_REPS:-2}
steps=${AB_STEPS:-5}
for rep in $(seq $reps); do
for v in "$@"; do
  unset JANUS_LIB
  envs=""
  case "$v" in
    default) ;;
    env:*) envs="${v#env:}"; envs="${envs//,/ }" ;;
    lib:*) l="${v#lib:}"
           case "$l" in *+env:*) envs="${l#*+env:}"; envs="${envs//,/ }"; l="${l%%+env:*}" ;; esac
           export JANUS_LIB="$l" ;;
  esac
  name=$(echo "$v" | tr -c 'A-Za-z0-9_=.\n' '_')
  out=gpurun_out/ab_${tag}_${name}_$rep
  env $envs timeout -k 10 300 python -u bench.py --steps $steps --warmup 2 --no-cpu-baseline --no-idle-latency \
    > $out.json 2> $out.err || { tail -5 $out.err; exit 1; }
  echo "$v $(python3 -c "
import json; d=json.load(open('$out.json'))
s=d['side_ms'] or {}
m=lambda k: round(sum(s.get(k,[0]))/max(len(s.get(k,[1])),1),1)
print(d['ms_per_step'], 'voc', m('vocoder'), 'dec', m('decoder'), 'conv', d['roofline']['avg_launch_ms'], 'yin', d.get('yin_dec_utts'), 'lpp', (d['roofline'].get('decoder') or {}).get('launches_per_position'))")"
done
done
