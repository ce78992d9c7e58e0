"""Summarise a rocprofv3 kernel trace: top kernels by total time.

python tools/rocprof_stats.py <kernel_stats.csv | results.db> [top_n] [--csv out.csv]
"""
import csv
import sqlite3
import sys


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        rows = c.execute("select name, count(*), sum(end - start), avg(end - start) from kernels "
                         "group by name").fetchall()
        return [{"Name": n, "Calls": k, "TotalDurationNs": t, "AverageNs": a} for n, k, t, a in rows]
    return list(csv.DictReader(open(path)))


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rows = load(args[0])
    top = int(args[1]) if len(args) > 1 else 20
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:top]:
        t = float(r["TotalDurationNs"])
        print(f"{t / 1e6:9.1f} ms {t / tot * 100:5.1f}% calls {int(r['Calls']):>6} "
              f"avg {float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:100]}")
    print("total ms", tot / 1e6)
    if "--csv" in sys.argv:
        out = sys.argv[sys.argv.index("--csv") + 1]
        with open(out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for r in rows:
                t = float(r["TotalDurationNs"])
                w.writerow([r["Name"], r["Calls"], int(t), float(r["AverageNs"]), round(t / tot * 100, 3)])


if __name__ == "__main__":
    main()
