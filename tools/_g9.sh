set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py -k "persistent" -x -q --timeout 300 --timeout-method thread > gpurun_out/t9.log 2>&1; rc=$?; tail -2 gpurun_out/t9.log; [ $rc -eq 0 ] || exit $rc
for lib in libjanus_hip_prev.so libjanus_hip.so libjanus_hip_prev.so libjanus_hip.so; do
JANUS_LIB=$lib timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-idle-latency > gpurun_out/b9.json 2> gpurun_out/b9.err || { tail -3 gpurun_out/b9.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/b9.json').read().strip().splitlines()[-1]);print('$lib', {k:d[k] for k in ['value','ms_per_step','side_ms']}); print(d['roofline']['decoder']['us_per_position'])"
done
