#!/bin/bash
set -o pipefail
for v in "X=1" "JANUS_WIDE128_WAVES=2" "JANUS_WIDE128_WAVES=8"; do
  env $v timeout -k 10 300 python -u -m pytest tests/test_vocoder_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "resunit or generator" > gpurun_out/ad_test.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ad_test.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ad_test.log)"
done
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in "X=1" "JANUS_WIDE128_WAVES=2" "JANUS_WIDE128_WAVES=8" "JANUS_LIB=libjanus_hip_old.so"; do
  tag=$(echo $v | tr '=' '_')
  env $v timeout -k 10 120 rocprofv3 --kernel-trace -d $root/gpurun_out/sd_$tag -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/sd_$tag.log 2>&1 || { tail -5 $root/gpurun_out/sd_$tag.log; exit 1; }
done
cd $root
python3 - <<'PY'
import csv, glob, re
for v in ("X_1", "JANUS_WIDE128_WAVES_2", "JANUS_WIDE128_WAVES_8", "JANUS_LIB_libjanus_hip_old.so"):
    f = glob.glob(f"gpurun_out/sd_{v}/**/*kernel_trace.csv", recursive=True)[0]
    fam = {}
    for r in csv.DictReader(open(f)):
        m = re.search(r"resunit(?:_wide)?(?:_lds)?_kernel<(\d+)", r["Kernel_Name"])
        if m:
            fam[m.group(1)] = fam.get(m.group(1), 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(v, {k: round(x, 2) for k, x in sorted(fam.items())})
PY
