#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_vocoder_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r_test.log 2>&1 || { tail -30 gpurun_out/r_test.log; exit 1; }
tail -1 gpurun_out/r_test.log
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for lib in default libjanus_hip_old.so; do
  if [ "$lib" = default ]; then unset JANUS_LIB; else export JANUS_LIB=$lib; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/vt_$lib -o run -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/vt_$lib.log 2>&1 || { tail -5 $root/gpurun_out/vt_$lib.log; exit 1; }
  f=$(find $root/gpurun_out/vt_$lib -name "*kernel_stats.csv" | head -1)
  echo "$lib: $(grep -E 'conv_post' $f | cut -c1-160)"
done
cd $root
unset JANUS_LIB
bash tools/gpu_abenv.sh post default JANUS_LIB=libjanus_hip_old.so
