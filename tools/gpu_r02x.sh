#!/bin/bash
set -o pipefail
for v in "JANUS_WIDE128_WAVES=8" "JANUS_WIDE64_WAVES=8" "JANUS_WIDE256_WAVES=16"; do
  env $v timeout -k 10 300 python -u -m pytest tests/test_vocoder_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "resunit or generator or family" > gpurun_out/x_test.log 2>&1 || { echo "FAIL $v"; grep -E "^FAILED|rms|assert" gpurun_out/x_test.log | head -5; continue; }
  echo "$v $(tail -1 gpurun_out/x_test.log)"
done
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in base w128 w64 w256; do
  case $v in w128) export JANUS_WIDE128_WAVES=8;; w64) export JANUS_WIDE64_WAVES=8;; w256) export JANUS_WIDE256_WAVES=16;; esac
  timeout -k 10 120 rocprofv3 --kernel-trace -d $root/gpurun_out/vx_$v -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/vx_$v.log 2>&1 || { tail -5 $root/gpurun_out/vx_$v.log; exit 1; }
  unset JANUS_WIDE128_WAVES JANUS_WIDE64_WAVES JANUS_WIDE256_WAVES
done
cd $root
python3 - <<'PY'
import csv, glob, re
for v in ("base", "w128", "w64", "w256"):
    f = glob.glob(f"gpurun_out/vx_{v}/**/*kernel_trace.csv", recursive=True)[0]
    fam = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        m = re.search(r"resunit(?:_wide)?(?:_lds)?_kernel<(\d+)", k)
        if m:
            fam[m.group(1)] = fam.get(m.group(1), 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(v, {k: round(x, 2) for k, x in sorted(fam.items())})
PY
