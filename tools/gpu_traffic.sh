#!/bin/bash
# PMC traffic of the vocoder conv launches (run via gpurun)
set -o pipefail
root=$(pwd)
mkdir -p $root/gpurun_out/traffic
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $root/gpurun_out/traffic/f -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/traffic/f.log 2>&1 || { tail -5 $root/gpurun_out/traffic/f.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $root/gpurun_out/traffic/w -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/traffic/w.log 2>&1 || { tail -5 $root/gpurun_out/traffic/w.log; exit 1; }
python3 $root/tools/vocoder_traffic.py --reduce $root/gpurun_out/traffic/f $root/gpurun_out/traffic/w $root/gpurun_out/traffic/traffic.json
