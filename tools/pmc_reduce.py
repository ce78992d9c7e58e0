"""Sum rocprofv3 --pmc counters per vocoder kernel family (or per kernel name with
--by-kernel) over one or more pass directories; prints JSON.

Normalisation (MI355X_MICROARCH.md, PMC units):
- SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles per wave; the stall split
  SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stall) +
  SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES is reported as fractions of SQ_WAVE_CYCLES.
- SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles summed over every SIMD; GRBM_GUI_ACTIVE is the
  active-cycle count summed over the 8 XCDs. The matrix-core busy fraction of the kernel's
  SIMDs over its run is therefore
      mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 4 * CUs)
  with CUs = the CUs the kernel ran on (--cus, default 256: a standalone run on the whole
  chip); it is <= 1 by construction. cycles_per_mfma = SQ_VALU_MFMA_BUSY_CYCLES /
  SQ_INSTS_MFMA checks the unit (16 for v_mfma_f32_16x16x32_f16).
- FETCH_SIZE (KB) is doubled: on gfx950 it reports half the bytes of a wide streaming read.

python tools/pmc_reduce.py DIR [DIR ...] [--by-kernel] [--cus N] [--filter S]
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from vocoder_traffic import family  # noqa: E402


def reduce_dirs(dirs, by_kernel=False, cus=256, filt=""):
    out = {}
    disp = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if filt and filt not in k:
                    continue
                key = k[:90] if by_kernel else str(family(k))
                if key == "None":
                    continue
                g = out.setdefault(key, {})
                c = r["Counter_Name"]
                v = float(r["Counter_Value"])
                if c == "FETCH_SIZE":
                    v *= 2.0
                g[c] = g.get(c, 0.0) + v
                disp.setdefault(key, {}).setdefault(c, set()).add((d, r["Dispatch_Id"]))
    for key, g in out.items():
        n = {c: len(s) for c, s in disp[key].items()}
        g["dispatches"] = max(n.values())
        if g.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in g:
            g["mfma_busy_frac"] = round(g["SQ_VALU_MFMA_BUSY_CYCLES"] / (g["GRBM_GUI_ACTIVE"] / 8 * 4 * cus), 4)
        if g.get("SQ_INSTS_MFMA") and "SQ_VALU_MFMA_BUSY_CYCLES" in g:
            g["cycles_per_mfma"] = round(g["SQ_VALU_MFMA_BUSY_CYCLES"] / g["SQ_INSTS_MFMA"], 2)
        if g.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in g:
                    g[c.lower() + "_frac"] = round(g[c] / g["SQ_WAVE_CYCLES"], 4)
        if g.get("SQ_LDS_IDX_ACTIVE"):
            g["lds_conflict_frac"] = round(g.get("SQ_LDS_BANK_CONFLICT", 0) / g["SQ_LDS_IDX_ACTIVE"], 4)
        if "FETCH_SIZE" in g:
            g["fetch_kb_per_dispatch"] = round(g["FETCH_SIZE"] / n["FETCH_SIZE"], 1)
    return out


def main():
    args = sys.argv[1:]
    by_kernel = "--by-kernel" in args
    cus, filt, dirs = 256, "", []
    i = 0
    while i < len(args):
        a = args[i]
        if a == "--cus":
            cus = int(args[i + 1]); i += 2; continue
        if a == "--filter":
            filt = args[i + 1]; i += 2; continue
        if not a.startswith("--"):
            dirs.append(a)
        i += 1
    print(json.dumps(reduce_dirs(dirs, by_kernel, cus, filt), indent=1))


if __name__ == "__main__":
    main()
