#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/stagger_diag.py 2>&1 | tee gpurun_out/stagger_diag.log
