set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_whisper_gpu.py -x -q -k "persistent_staggered or free_running_decode_base" --timeout 200 --timeout-method thread > gpurun_out/t6.log 2>&1; rc=$?; tail -2 gpurun_out/t6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-idle-latency > gpurun_out/b6.json 2> gpurun_out/b6.err || { tail -3 gpurun_out/b6.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/b6.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ['value','ms_per_step','side_ms','yin_dec_utts']}); print(d['roofline']['decoder']['us_per_position'])"
