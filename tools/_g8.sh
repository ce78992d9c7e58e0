set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pipe.log 2>&1; rc=$?; tail -2 gpurun_out/t_pipe.log; [ $rc -eq 0 ] || exit $rc
for v in voc hi; do
JANUS_CONT_ENCODE=$v timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-idle-latency > gpurun_out/b8_$v.json 2> gpurun_out/b8_$v.err || { tail -3 gpurun_out/b8_$v.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/b8_$v.json').read().strip().splitlines()[-1]);print('$v', {k:d[k] for k in ['value','ms_per_step','side_ms','yin_dec_utts']}); print(d['roofline']['decoder']['us_per_position'])"
done
