#!/bin/bash
# SQ counters + fetch per decoder kernel (decoder alone, 16 CUs per XCD, 64 positions); run via gpurun
set -o pipefail
root=$(pwd)
mkdir -p $root/gpurun_out/dpmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES -d $root/gpurun_out/dpmc/p1 -o run --output-format csv -- python3 $root/tools/decoder_probe.py --per-xcd 16 --beside 0 --reps 1 --max-length 64 > $root/gpurun_out/dpmc/p1.log 2>&1 || { tail -5 $root/gpurun_out/dpmc/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $root/gpurun_out/dpmc/p2 -o run --output-format csv -- python3 $root/tools/decoder_probe.py --per-xcd 16 --beside 0 --reps 1 --max-length 64 > $root/gpurun_out/dpmc/p2.log 2>&1 || { tail -5 $root/gpurun_out/dpmc/p2.log; exit 1; }
cd $root
python3 - <<'PY'
import csv, glob
tot = {}
for d in ("p1", "p2"):
    f = glob.glob(f"gpurun_out/dpmc/{d}/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        g = tot.setdefault(k, {})
        c = r["Counter_Name"]
        g[c] = g.get(c, 0.0) + float(r["Counter_Value"])
        g.setdefault("_d", set()).add((d, r["Dispatch_Id"]))
for k, g in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:12]:
    n = len([x for x in g["_d"] if x[0] == "p1"])
    wc = g.get("SQ_WAVE_CYCLES", 1)
    print(f"{k:60s} n={n:5d} waves/disp={g.get('SQ_WAVES',0)/max(n,1):7.0f} wait={g.get('SQ_WAIT_ANY',0)/wc:.2f} "
          f"issue_stall={g.get('SQ_WAIT_INST_ANY',0)/wc:.2f} active={g.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} "
          f"valu/wave={g.get('SQ_INSTS_VALU',0)/max(g.get('SQ_WAVES',1),1):.0f} lds/wave={g.get('SQ_INSTS_LDS',0)/max(g.get('SQ_WAVES',1),1):.0f} "
          f"fetchKB/disp={2*g.get('FETCH_SIZE',0)/max(len([x for x in g['_d'] if x[0]=='p2']),1):.0f}")
PY
