#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_vocoder_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "resunit or generator or family" > gpurun_out/y_test.log 2>&1 || { tail -30 gpurun_out/y_test.log; exit 1; }
tail -1 gpurun_out/y_test.log
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in default libjanus_hip_old.so; do
  if [ $v = default ]; then unset JANUS_LIB; else export JANUS_LIB=$v; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d $root/gpurun_out/vy_$v -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/vy_$v.log 2>&1 || { tail -5 $root/gpurun_out/vy_$v.log; exit 1; }
done
unset JANUS_LIB
cd $root
python3 - <<'PY'
import csv, glob, re
for v in ("default", "libjanus_hip_old.so"):
    f = glob.glob(f"gpurun_out/vy_{v}/**/*kernel_trace.csv", recursive=True)[0]
    fam = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        m = re.search(r"resunit(?:_wide)?(?:_lds)?_kernel<(\d+)", k)
        if m:
            fam[m.group(1)] = fam.get(m.group(1), 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(v, {k: round(x, 2) for k, x in sorted(fam.items())})
PY
bash tools/gpu_abenv.sh np default JANUS_LIB=libjanus_hip_old.so
