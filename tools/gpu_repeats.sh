#!/bin/bash
# bench line repeated on one box (spread of the headline) + the back-to-back step (whole-GPU roofline)
set -o pipefail
mkdir -p gpurun_out/rep
for i in 1 2 3; do
  JANUS_OVERLAP_TIMING=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/rep/b$i.json 2> gpurun_out/rep/b$i.err || { tail -5 gpurun_out/rep/b$i.err; exit 1; }
  tail -1 gpurun_out/rep/b$i.json | cut -c1-200
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --overlap 0 > gpurun_out/rep/b2b.json 2> gpurun_out/rep/b2b.err || { tail -5 gpurun_out/rep/b2b.err; exit 1; }
tail -1 gpurun_out/rep/b2b.json | cut -c1-200
