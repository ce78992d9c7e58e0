#!/bin/bash
# r04: staggered (continuous-batching) decoder — parity tests, then same-box bench pairs
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/r04d
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py tests/test_pipeline_gpu.py -x -v --timeout 300 \
  --timeout-method thread -k "stagger or shared" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for rep in 1 2; do
for sg in 0 1; do
  timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --fallback-steps 0 --no-idle-latency --stagger $sg \
    > $out/bench_s${sg}_$rep.log 2>&1 || { tail -20 $out/bench_s${sg}_$rep.log; exit 1; }
  tail -1 $out/bench_s${sg}_$rep.log > $out/bench_s${sg}_$rep.json
  python3 -c "
import json; d=json.load(open('$out/bench_s${sg}_$rep.json')); print('stagger $sg', d['ms_per_step'], d['value'], d['step_ms'], d['side_ms'], d['roofline']['decoder']['us_per_position'], d['roofline']['decoder']['launches_per_position'])"
done
done
