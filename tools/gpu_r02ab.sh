#!/bin/bash
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_vocoder_gpu.py tests/test_kernels_gpu.py tests/test_whisper_gpu.py -x -q --timeout 300 --timeout-method thread -k "resunit or generator or family or decode or seek or end_to_end" > gpurun_out/ab_test.log 2>&1 || { tail -30 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in default libjanus_hip_old.so; do
  if [ $v = default ]; then unset JANUS_LIB; else export JANUS_LIB=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/sb_$v -o run --output-format csv -- python3 $root/tools/decoder_probe.py --per-xcd 16 --beside 0 --reps 2 --max-length 64 > $root/gpurun_out/sb_$v.log 2>&1 || { tail -5 $root/gpurun_out/sb_$v.log; exit 1; }
  f=$(find $root/gpurun_out/sb_$v -name "*kernel_stats.csv" | head -1)
  echo "$v: $(grep -E 'logits_partial' $f | cut -d, -f2-4)"
  timeout -k 10 120 rocprofv3 --kernel-trace -d $root/gpurun_out/sv_$v -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/sv_$v.log 2>&1 || { tail -5 $root/gpurun_out/sv_$v.log; exit 1; }
done
unset JANUS_LIB
cd $root
python3 - <<'PY'
import csv, glob, re
for v in ("default", "libjanus_hip_old.so"):
    f = glob.glob(f"gpurun_out/sv_{v}/**/*kernel_trace.csv", recursive=True)[0]
    fam = {}
    for r in csv.DictReader(open(f)):
        m = re.search(r"resunit(?:_wide)?(?:_lds)?_kernel<(\d+)", r["Kernel_Name"])
        if m:
            fam[m.group(1)] = fam.get(m.group(1), 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(v, {k: round(x, 2) for k, x in sorted(fam.items())})
PY
bash tools/gpu_abenv.sh sb default JANUS_LIB=libjanus_hip_old.so
