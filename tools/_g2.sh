set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py -k "persistent_staggered" -x -v --timeout 300 --timeout-method thread > gpurun_out/t_pers.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/t_pers.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pipe.log 2>&1; rc=$?; tail -3 gpurun_out/t_pipe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --fallback-steps 0 --first-window-steps 0 > gpurun_out/b2.json 2> gpurun_out/b2.err; rc=$?; tail -3 gpurun_out/b2.err; python -c "
import json;d=json.loads(open('gpurun_out/b2.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ['value','ms_per_step','side_ms','windows_decoded','seek_windows_extra','p50_latency_ms','yin_dec_utts','decoder_calls_per_step']}); print(d['roofline']['decoder'])"; exit $rc
