#!/bin/bash
# PMC traffic of the vocoder conv launches (run via gpurun): tools/gpu_traffic.sh [tag]
# (JANUS_LIB selects an A/B build)
set -o pipefail
root=$(pwd)
tag=${1:-traffic}
out=$root/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/f -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $out/f.log 2>&1 || { tail -5 $out/f.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/w -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $out/w.log 2>&1 || { tail -5 $out/w.log; exit 1; }
python3 $root/tools/vocoder_traffic.py --reduce $out/f $out/w $out/traffic.json
