"""Per-kernel PMC summary of tools/gpu_pmc.sh passes.

python tools/pmc_summary.py gpurun_out/<tag> [name_filter]
-> for every kernel (matching the filter): dispatches and the per-dispatch mean of every
   counter collected in any pass (FETCH_SIZE doubled per MI355X_MICROARCH.md 'HBM').
"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if filt and filt not in name:
                continue
            c = r["Counter_Name"]
            v = float(r["Counter_Value"])
            if c == "FETCH_SIZE":
                v *= 2.0
            vals[name][c] += v
            disp[name][c].add(r["Dispatch_Id"])
    for name in sorted(vals):
        print(name[:110])
        for c in sorted(vals[name]):
            n = len(disp[name][c])
            print(f"   {c:28s} {vals[name][c] / n:16.1f}  (n={n})")


if __name__ == "__main__":
    main()
