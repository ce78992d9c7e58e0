set -o pipefail
for v in 0 131072; do
JANUS_DEC_PATH_FLAGS=$v timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-idle-latency > gpurun_out/b7_$v.json 2> gpurun_out/b7_$v.err || { tail -3 gpurun_out/b7_$v.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/b7_$v.json').read().strip().splitlines()[-1]);print('$v', {k:d[k] for k in ['value','ms_per_step','side_ms','yin_dec_utts']}); print(d['roofline']['decoder']['us_per_position'])"
done
