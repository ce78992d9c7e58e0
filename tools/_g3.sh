set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py -k "persistent_staggered" -x -v --timeout 300 --timeout-method thread > gpurun_out/t_pers.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/t_pers.log | tail -15; [ $rc -eq 0 ] || exit $rc
for v in 0 65536; do
JANUS_DEC_PATH_FLAGS=$v timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-idle-latency > gpurun_out/b3_$v.json 2> gpurun_out/b3_$v.err || { tail -3 gpurun_out/b3_$v.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/b3_$v.json').read().strip().splitlines()[-1]);print('$v', {k:d[k] for k in ['value','ms_per_step','side_ms','yin_dec_utts']}); print(d['roofline']['decoder']['us_per_position'])"
done
