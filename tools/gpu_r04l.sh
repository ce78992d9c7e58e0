#!/bin/bash
# r04: decoder launch-geometry knobs at 128 rows (staggered step), decoder side isolated
# (no YIN on its CUs): one bench run per knob, baseline first and last
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04l
mkdir -p $out
export JANUS_YIN_DEC_UTTS=0
for knob in ${KNOBS:-base}; do
  tag=${knob//=/_}
  if [ "${knob:0:4}" = base ]; then envs=""; else envs="$knob"; fi
  env $envs timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency \
    > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['side_ms']['decoder'], d['roofline']['decoder']['us_per_position'])"
done
for xs in ${FBXS:-}; do
  JANUS_FB_XSPLITS=$xs timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 1 > $out/fb_xs$xs.log 2>&1 || { tail -20 $out/fb_xs$xs.log; exit 1; }
  tail -1 $out/fb_xs$xs.log > $out/fb_xs$xs.json
  python3 -c "
import json; d=json.load(open('$out/fb_xs$xs.json')); print('fb_xs$xs', d['xrt_with_fallback'], d['fallback']['step_ms'])"
done
