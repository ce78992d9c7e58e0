#!/bin/bash
# r04: fallback re-decodes on the whole GPU (JANUS_FB_FULL=1, default) vs the decoder's CUs:
# parity, then two same-box pairs of the bench's fallback leg
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04k
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "fallback" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
for ff in 1 0; do
  for xs in ${XS:-4}; do
  tag=ff${ff}_xs${xs}_$rep
  JANUS_FB_FULL=$ff JANUS_FB_XSPLITS=$xs timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 1 \
    > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['xrt_with_fallback'], d['fallback']['step_ms'])"
  done
done
done
