#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_vocoder_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "resunit or generator or family" > gpurun_out/v_test.log 2>&1 || { tail -30 gpurun_out/v_test.log; exit 1; }
tail -1 gpurun_out/v_test.log
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for lib in default libjanus_hip_old.so; do
  if [ "$lib" = default ]; then unset JANUS_LIB; else export JANUS_LIB=$lib; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d $root/gpurun_out/vt_$lib -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/vt_$lib.log 2>&1 || { tail -5 $root/gpurun_out/vt_$lib.log; exit 1; }
done
cd $root
unset JANUS_LIB
python3 - <<'PY'
import csv, glob
for lib in ("default", "libjanus_hip_old.so"):
    f = glob.glob(f"gpurun_out/vt_{lib}/**/*kernel_trace.csv", recursive=True)[0]
    fam = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "resunit_kernel<" in k:
            c = k.split("<")[1].split(",")[0]
            fam[c] = fam.get(c, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(lib, {k: round(v, 2) for k, v in fam.items()})
PY
bash tools/gpu_abenv.sh nb default JANUS_LIB=libjanus_hip_old.so
