"""Cross-check of the bench line's roofline against the rocprofv3 kernel trace of the same
command: the vocoder conv/unit launches' average duration in kernel_stats.csv vs the
line's roofline.avg_launch_ms (HIP events). The encoder-stem convs (conv_kernel<..., 0, 2>)
and the weight-pack kernels are not vocoder launches and are excluded.

python tools/conv_avg.py <kernel_stats.csv | results.db> bench_line.json

Since r05 the staggered step renders a few utterances on the decoder's CUs with a second
vocoder context (JANUS_VOC_DEC_UTTS): its launches carry a few rows and the line's roofline
(the main context's HIP events) leaves them out. Given the trace database, only the
launches on the stream that carries the main context (the largest total grid) are
averaged; the CSV form averages every vocoder launch.
"""
import sqlite3
import csv
import json
import re
import sys


def is_vocoder_conv(name):
    if "pack_kernel" in name:
        return False
    if re.search(r"conv_kernel<[^>]*, 2>", name):
        return False   # Whisper encoder stem (GELU + positional embedding epilogue)
    return ("conv_kernel<" in name or "resunit_wide_kernel<" in name
            or "resunit_wide_lds_kernel<" in name or "resunit_kernel<" in name)


def main_stream_launches(db):
    c = sqlite3.connect(db)
    rows = [r for r in c.execute("select name, stream_id, grid_x * grid_y * grid_z, end - start from kernels")
            if is_vocoder_conv(r[0])]
    grid = {}
    for _, sid, g, _ in rows:
        grid[sid] = grid.get(sid, 0) + g
    main_sid = max(grid, key=grid.get)
    durs = [d for _, sid, _, d in rows if sid == main_sid]
    return len(durs), float(sum(durs))


def main():
    if sys.argv[1].endswith(".db"):
        calls, ns = main_stream_launches(sys.argv[1])
    else:
        rows = [r for r in csv.DictReader(open(sys.argv[1])) if is_vocoder_conv(r["Name"])]
        calls = sum(int(r["Calls"]) for r in rows)
        ns = sum(float(r["TotalDurationNs"]) for r in rows)
    line = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    rf = line["roofline"]
    prof_ms = ns / max(calls, 1) / 1e6
    flops = rf["flops_per_launch"]
    out = {"rocprof_launches": calls, "rocprof_avg_launch_ms": round(prof_ms, 4),
           "line_launches": rf["launches"], "line_avg_launch_ms": rf["avg_launch_ms"],
           "ratio_line_over_rocprof": round(rf["avg_launch_ms"] / prof_ms, 4),
           "rocprof_tflops": round(flops / (prof_ms * 1e-3) / 1e12, 1),
           "rocprof_frac": round(flops / (prof_ms * 1e-3) / 1e12 / 2500.0, 4),
           "line_frac": rf["frac"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
