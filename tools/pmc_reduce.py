"""Sum rocprofv3 --pmc counters per vocoder kernel family (and per kernel name with
--by-kernel) over one or more pass directories; prints JSON. Stall accounting per the
MI355X guide: SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stall)
+ SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES; SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CU_CYCLES ~=
matrix-core busy fraction of the CUs' busy time.

python tools/pmc_reduce.py DIR [DIR ...] [--by-kernel]
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from vocoder_traffic import family  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    by_kernel = "--by-kernel" in sys.argv
    out = {}
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                key = k[:90] if by_kernel else str(family(k))
                if key == "None":
                    continue
                g = out.setdefault(key, {})
                c = r["Counter_Name"]
                g[c] = g.get(c, 0.0) + float(r["Counter_Value"])
    for g in out.values():
        if g.get("SQ_BUSY_CU_CYCLES"):
            g["mfma_busy_frac"] = round(g.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / g["SQ_BUSY_CU_CYCLES"], 4)
        if g.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in g:
                    g[c.lower() + "_frac"] = round(g[c] / g["SQ_WAVE_CYCLES"], 4)
        if g.get("SQ_LDS_IDX_ACTIVE"):
            g["lds_conflict_frac"] = round(g.get("SQ_LDS_BANK_CONFLICT", 0) / g["SQ_LDS_IDX_ACTIVE"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
