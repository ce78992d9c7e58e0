#!/bin/bash
# round 2: GPU test suite + free-running decode parity measurement
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r02a_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r02a_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/decode_parity.py --model base.en --n 6 > gpurun_out/r02a_parity.json 2> gpurun_out/r02a_parity.err
rc=$?
cat gpurun_out/r02a_parity.json
exit $rc
