#!/bin/bash
# decoder kernels alone vs beside the vocoder (16 CUs per XCD)
set -o pipefail
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for bes in 0 1; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/dp$bes -o run -- python3 $root/tools/decoder_probe.py --per-xcd 16 --beside $bes --reps 2 > $root/gpurun_out/dp$bes.log 2>&1 || { tail -20 $root/gpurun_out/dp$bes.log; exit 1; }
grep '{' $root/gpurun_out/dp$bes.log
f=$(find $root/gpurun_out/dp$bes -name "*.db" | head -1)
python3 $root/tools/rocprof_stats.py "$f" 30 --csv $root/gpurun_out/dp$bes/kernel_stats.csv | head -32
done
