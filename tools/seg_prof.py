"""Phase timeline of the persistent decoder segments (dec_persist.hip) inside the headline
staggered step: a JANUS_PHASE_PROF build stamps the real-time clock (100 MHz) per block at
kernel start, at every grid barrier's arrival / release and before the exit, for the
launches of one layer (JANUS_SEG_PROF=l; the buffer keeps the last such launch).

usage: JANUS_LIB=libjanus_hip_prof.so JANUS_SEG_PROF=2 python tools/seg_prof.py [bench args]
(build: make -C janus_amd/csrc OUT=../libjanus_hip_prof.so OBJDIR=../../build/obj_prof
 DEFS=-DJANUS_PHASE_PROF)
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summarize(p, nbar):
    """p: [blocks][48] stamps of one launch (10 ns ticks): [0] start, [2e-1] / [2e] barrier e
    arrival / release, [15] end, marks of phase p at [18 + 3 (p - 1) + i]."""
    p = p[p[:, 0] > 0]
    if len(p) == 0:
        return None
    us = lambda v: round(float(v) / 100.0, 2)  # noqa: E731
    t0 = p[:, 0].min()
    out = {"blocks": int(len(p)), "span_us": us(p[:, 15].max() - t0),
           "start_skew_us": us(p[:, 0].max() - t0), "phases": []}
    prev = p[:, 0]
    for e in range(1, nbar + 2):
        arr = p[:, 15] if e == nbar + 1 else p[:, 2 * e - 1]
        inner = [p[:, 18 + 3 * (e - 1) + i] for i in range(3)] if e <= 5 else [p[:, 0] * 0] * 3
        ph = {"compute_med_us": us(np.median(arr - prev)), "compute_max_us": us((arr - prev).max()),
              # wave 0's marks inside the phase, from the phase start (medians)
              "marks_med_us": [us(np.median(m - prev)) if (m > 0).all() else None for m in inner],
              "arrive_skew_us": us(arr.max() - arr.min()),
              "arrive_last_us": us(arr.max() - t0)}
        if e <= nbar:
            rel = p[:, 2 * e]
            ph["last_arrive_to_first_release_us"] = us(rel.min() - arr.max())
            ph["release_skew_us"] = us(rel.max() - rel.min())
            prev = rel
        out["phases"].append(ph)
    return out


def main():
    assert os.environ.get("JANUS_SEG_PROF") is not None and os.environ.get("JANUS_LIB"), __doc__
    argv = sys.argv[1:] or ["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-idle-latency"]
    sys.argv = [os.path.join(ROOT, "bench.py")] + argv
    import bench
    from janus_amd import _native
    bench.main()
    fn = _native.lib().janus_debug_seg_read
    fn.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
    buf = np.zeros((768, 48), dtype=np.int64)
    n = fn(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), 768)
    assert n == 768, n
    res = {"layer": int(os.environ["JANUS_SEG_PROF"]),
           "seg_a": summarize(buf[:256], 1), "seg_b": summarize(buf[256:512], 4),
           "layer_kernel": summarize(buf[512:], 7)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
