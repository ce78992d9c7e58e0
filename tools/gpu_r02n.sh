#!/bin/bash
set -o pipefail
bash tools/gpu_abenv.sh ln default "JANUS_LN_PROLOGUE=1" "JANUS_FUSED_LN=1" || exit 1
bash tools/gpu_r02m.sh
