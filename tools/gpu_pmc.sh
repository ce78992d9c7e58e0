#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only) over kbench shapes.
# usage (via gpurun): bash tools/gpu_pmc.sh <tag> <kbench args...>
set -o pipefail
tag=$1; shift
root=$(pwd)
mkdir -p $root/gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $root/gpurun_out/$tag/counters.txt 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $root/gpurun_out/$tag/p$i -o run --output-format csv -- python3 $root/${SCRIPT:-tools/kbench.py} "$@" > $root/gpurun_out/$tag/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $root/gpurun_out/$tag/p$i.log; exit 1; }
done
echo done
