#!/bin/bash
# r05: the tests this round touched (staggered ABI check, fallback through the staggered
# step, base.en streaming parity); bench with "bench" as $2
set -o pipefail
out=gpurun_out/${1:-r05a}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_pipeline_gpu.py tests/test_streaming_gpu.py "tests/test_whisper_gpu.py::test_staggered_offset_past_stand_is_rejected" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
[ "$2" == "bench" ] || exit 0
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print({k: d.get(k) for k in ('value','ms_per_step','p50_latency_ms','p50_latency_ms_overlapped','xrt_with_fallback','seek_windows_extra','side_ms')})
print(d.get('fallback')); print(d.get('overlapped'))"
