#!/bin/bash
# r04: vocoder launch knobs re-swept in the staggered step (YIN split pinned at 40 so the
# vocoder side is comparable): one bench run per knob, baseline first and last
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/vocknobs
mkdir -p $out
export JANUS_YIN_DEC_UTTS=40
for knob in ${KNOBS:-base}; do
  tag=${knob//=/_}
  if [ "${knob:0:4}" = base ]; then envs=""; else envs="$knob"; fi
  env $envs timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency \
    > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['side_ms']['vocoder'], d['roofline']['avg_launch_ms'])"
done
