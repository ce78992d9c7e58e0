#!/bin/bash
# PMC summaries (run via gpurun): the greedy decoder at the headline shape (128 rows,
# 16 CUs per XCD, alone, 64 positions) with the persistent segments on and off, and the
# vocoder families (standalone 64 x 30 s forward), counters normalised by tools/pmc_reduce.py
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/${1:-pmc}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
DEC="python3 $root/tools/decoder_probe.py --per-xcd 16 --beside 0 --reps 1 --max-length 64 --rows 128 --xsplits 1"
for P in 1 0; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE -d $out/dec$P/p1 -o run --output-format csv -- $DEC --persistent $P > $out/dec$P.p1.log 2>&1 || { tail -5 $out/dec$P.p1.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/dec$P/p2 -o run --output-format csv -- $DEC --persistent $P > $out/dec$P.p2.log 2>&1 || { tail -5 $out/dec$P.p2.log; exit 1; }
  python3 $root/tools/pmc_reduce.py $out/dec$P/p1 $out/dec$P/p2 --by-kernel --cus 128 > $out/decoder_persistent$P.json
done
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $out/voc/p1 -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $out/voc.p1.log 2>&1 || { tail -5 $out/voc.p1.log; exit 1; }
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES -d $out/voc/p2 -o run --output-format csv -- python3 $root/tools/vocoder_traffic.py > $out/voc.p2.log 2>&1 || { tail -5 $out/voc.p2.log; exit 1; }
python3 $root/tools/pmc_reduce.py $out/voc/p1 $out/voc/p2 --cus 256 > $out/vocoder_families.json
grep -h '"decoder_ms"' $out/dec1.p1.log $out/dec0.p1.log || true
python3 - <<PY
import json
for P in (1, 0):
    d = json.load(open("$out/decoder_persistent%d.json" % P))
    print("persistent", P)
    for k, v in sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:10]:
        print("  %-60s n=%5d wait=%.2f issue=%.2f active=%.2f fetchKB=%s" % (k[:60], v["dispatches"],
              v.get("sq_wait_any_frac", 0), v.get("sq_wait_inst_any_frac", 0), v.get("sq_active_inst_any_frac", 0),
              v.get("fetch_kb_per_dispatch")))
v = json.load(open("$out/vocoder_families.json"))
for k, g in v.items():
    print(k, {x: g.get(x) for x in ("mfma_busy_frac", "cycles_per_mfma", "sq_wait_any_frac", "sq_wait_inst_lds_frac", "lds_conflict_frac", "fetch_kb_per_dispatch")})
PY
