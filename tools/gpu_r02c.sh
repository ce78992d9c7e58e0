#!/bin/bash
# round 2: GPU suite (new parity tests) + one bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread \
  > gpurun_out/r02c_pytest.log 2>&1
rc=$?
grep -E "passed|failed|error|identical|rel RMS|rms" gpurun_out/r02c_pytest.log | tail -25
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r02c_bench.json 2> gpurun_out/r02c_bench.err
rc=$?
cat gpurun_out/r02c_bench.json
exit $rc
