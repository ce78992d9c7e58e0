#!/bin/bash
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_whisper_gpu.py tests/test_pipeline_gpu.py tests/test_streaming_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ac_test.log 2>&1 || { tail -30 gpurun_out/ac_test.log; exit 1; }
tail -1 gpurun_out/ac_test.log
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in default libjanus_hip_old.so; do
  if [ $v = default ]; then unset JANUS_LIB; else export JANUS_LIB=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/sc_$v -o run --output-format csv -- python3 $root/tools/decoder_probe.py --per-xcd 16 --beside 0 --reps 2 --max-length 64 > $root/gpurun_out/sc_$v.log 2>&1 || { tail -5 $root/gpurun_out/sc_$v.log; exit 1; }
  f=$(find $root/gpurun_out/sc_$v -name "*kernel_stats.csv" | head -1)
  echo "$v: $(grep -E 'logits_partial' $f | cut -d, -f2-4)"
done
unset JANUS_LIB
cd $root
bash tools/gpu_abenv.sh sc default JANUS_LIB=libjanus_hip_old.so
