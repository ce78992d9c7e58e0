#!/bin/bash
# r04: keep-all staging default (traffic + vocoder parity), YIN split at 2 cross-attention
# key splits, decoder skinny row-split threshold
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04j
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_vocoder_gpu.py -x -q --timeout 200 --timeout-method thread \
  > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
bash tools/gpu_traffic.sh traffic_r04 || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/traffic_r04/traffic.json')); print('traffic', round(d['traffic_over_algorithmic'],3), {k: round(v['traffic_over_algorithmic'],3) for k,v in d['by_family'].items()})"
for cfg in "24 0" "32 0" "40 0" "32 512" "32 4096"; do
  set -- $cfg
  tag=yd$1_ms$2
  if [ $2 = 0 ]; then unset JANUS_DEC_MSPLIT_N; else export JANUS_DEC_MSPLIT_N=$2; fi
  JANUS_YIN_DEC_UTTS=$1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency \
    > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log > $out/$tag.json
  python3 -c "
import json; d=json.load(open('$out/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'], d['roofline']['decoder']['us_per_position'])"
done
