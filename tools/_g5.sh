set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_bench_config_gpu.py -x -q -s --timeout 800 --timeout-method thread > gpurun_out/t_benchcfg.log 2>&1; rc=$?; grep -E "windows|row|bench rows|passed|failed" gpurun_out/t_benchcfg.log | tail -20; [ $rc -eq 0 ] || exit $rc
for ov in 16 20; do
timeout -k 10 400 python -u bench.py --overlap $ov --steps 4 --warmup 1 --no-cpu-baseline --no-idle-latency > gpurun_out/b5_$ov.json 2> gpurun_out/b5_$ov.err || { tail -3 gpurun_out/b5_$ov.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/b5_$ov.json').read().strip().splitlines()[-1]);print('$ov', {k:d[k] for k in ['value','ms_per_step','side_ms','yin_dec_utts']}); print(d['roofline']['decoder']['us_per_position'])"
done
bash tools/gpu_traffic.sh traffic_r06 && cat gpurun_out/traffic_r06/traffic.json | head -c 1500
