#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_streaming_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r02e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r02e_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/stream_bench.py --streams 16 --seconds 30 --max-length 448 > gpurun_out/r02e_stream.json 2> gpurun_out/r02e_stream.err || exit $?
cat gpurun_out/r02e_stream.json
timeout -k 10 300 python -u tools/stream_bench.py --streams 16 --seconds 30 --max-length 96 > gpurun_out/r02e_stream96.json 2> gpurun_out/r02e_stream96.err || exit $?
cat gpurun_out/r02e_stream96.json
