#!/bin/bash
# Decoder attention A/B (run via gpurun): kernel tests, cold-cache microbenchmarks of the
# current and previous kernels, bench step.
set -o pipefail
mkdir -p gpurun_out
o=gpurun_out/attn
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > $o/kt.log 2>&1 || { tail -30 $o/kt.log; exit 1; }
tail -1 $o/kt.log
timeout -k 10 200 python tools/kbench.py --xattn > $o/xattn_line.log 2>&1 || { tail -20 $o/xattn_line.log; exit 1; }
JANUS_XATTN_FRAG=1 timeout -k 10 200 python tools/kbench.py --xattn > $o/xattn_frag.log 2>&1 || { tail -20 $o/xattn_frag.log; exit 1; }
timeout -k 10 200 python tools/kbench.py --dec > $o/dec_head.log 2>&1 || { tail -20 $o/dec_head.log; exit 1; }
JANUS_DEC_SPLIT=1 timeout -k 10 200 python tools/kbench.py --dec > $o/dec_split.log 2>&1 || { tail -20 $o/dec_split.log; exit 1; }
for f in xattn_line xattn_frag dec_head dec_split; do echo "== $f"; cat $o/$f.log; done
timeout -k 10 400 python -u -m pytest tests/test_whisper_gpu.py -x -q --timeout 120 --timeout-method thread > $o/wt.log 2>&1 || { tail -30 $o/wt.log; exit 1; }
tail -1 $o/wt.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $o/bench.log
