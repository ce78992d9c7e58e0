#!/bin/bash
set -o pipefail
JANUS_NARROW_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_vocoder_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "resunit or generator or family" > gpurun_out/w_test.log 2>&1 || { tail -30 gpurun_out/w_test.log; exit 1; }
tail -1 gpurun_out/w_test.log
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for nw in 4 8; do
  JANUS_NARROW_WAVES=$nw timeout -k 10 120 rocprofv3 --kernel-trace -d $root/gpurun_out/vw_$nw -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $root/gpurun_out/vw_$nw.log 2>&1 || { tail -5 $root/gpurun_out/vw_$nw.log; exit 1; }
done
cd $root
python3 - <<'PY'
import csv, glob
for nw in (4, 8):
    f = glob.glob(f"gpurun_out/vw_{nw}/**/*kernel_trace.csv", recursive=True)[0]
    fam = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "resunit_kernel<" in k:
            key = ",".join(k.split("<")[1].split(",")[:2])
            fam[key] = fam.get(key, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(nw, {k: round(v, 2) for k, v in sorted(fam.items())}, round(sum(fam.values()), 2))
PY
bash tools/gpu_abenv.sh nw default JANUS_NARROW_WAVES=8
