#!/bin/bash
# round 2: free-running decode parity (decoder-only and end-to-end) at full length
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/decode_parity.py --model base.en --n 8 --e2e > gpurun_out/r02b_base.json 2> gpurun_out/r02b_base.err || exit $?
timeout -k 10 500 python -u tools/decode_parity.py --model tiny.en --n 16 --seed 3 --e2e > gpurun_out/r02b_tiny.json 2> gpurun_out/r02b_tiny.err
