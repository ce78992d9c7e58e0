"""Phase profile of one fused ResBlock1 unit launch (JANUS_PHASE_PROF build of the ring
kernel, resunit_wide.hip): runs one standalone 64 x 30 s vocoder forward with
JANUS_LIB=libjanus_hip_prof.so JANUS_PHASE_PROF=C,k,d and prints per-phase medians
(shader clocks, wave 0 of each block), the shader clock rate (clock64 against the 100 MHz
real-time counter) and how the blocks that share a CU overlap in time.
usage: JANUS_LIB=libjanus_hip_prof.so JANUS_PHASE_PROF=128,7,3 python tools/phase_prof.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from janus_amd import _native  # noqa: E402
from janus_amd.vocoder import VocoderEngine, emotion_id  # noqa: E402

PHASES = ["stage", "c1_loop", "c1_sync", "c1_epi", "c2_loop", "c2_sync", "epilogue"]


def main():
    B, F = 64, 2584
    eng = VocoderEngine()
    lat = eng.frontend([b"(relaxed) prof %d" % i for i in range(B)], [emotion_id("relaxed")] * B, F)
    eng.forward(lat)
    torch.cuda.synchronize()
    lib = _native.lib()
    fn = lib.janus_debug_phase_read
    fn.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
    cap = 1 << 20
    buf = np.zeros((cap, 16), dtype=np.int64)
    n = fn(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), cap)
    assert n > 0, n
    p = buf[:n]
    t = p[:, :8].astype(np.float64)
    d = np.diff(t, axis=1)
    tot = t[:, 7] - t[:, 0]
    wall = (p[:, 9] - p[:, 8]).astype(np.float64)
    ok = wall > 0
    ghz = float(np.median(tot[ok] / wall[ok] * 0.1))
    out = {"unit": os.environ.get("JANUS_PHASE_PROF"), "blocks": int(n), "shader_ghz": round(ghz, 3),
           "median_cycles": {ph: float(np.median(d[:, i])) for i, ph in enumerate(PHASES)},
           "mean_cycles": {ph: round(float(np.mean(d[:, i])), 1) for i, ph in enumerate(PHASES)},
           "median_total": float(np.median(tot))}
    # co-residency: blocks on one CU (XCC, SE/SH/CU fields of HW_ID), real-time overlap
    hw = p[:, 10]
    cu = (p[:, 11] & 0xF) * 4096 + ((hw >> 8) & 0xFF)
    start, end = p[:, 8], p[:, 9]
    span = float(end.max() - start.min()) / 100.0  # us
    keys, counts = np.unique(cu, return_counts=True)
    out["cus_seen"] = int(len(keys))
    out["blocks_per_cu_median"] = float(np.median(counts))
    out["launch_us"] = round(span, 1)
    # for a few CUs: how many blocks are live at each block's start, and start skew of
    # blocks that start within 2 us of each other (lockstep if skew ~ 0)
    live = []
    skews = []
    for k in keys[:64]:
        idx = np.where(cu == k)[0]
        s, e = start[idx], end[idx]
        order = np.argsort(s)
        s, e = s[order], e[order]
        for i in range(len(s)):
            live.append(int(np.sum((s <= s[i]) & (e > s[i]))))
        ends = np.sort(e)
        gaps = np.diff(np.sort(s)) / 100.0
        skews.extend(gaps.tolist())
    out["live_blocks_at_start_hist"] = {str(v): int(c) for v, c in zip(*np.unique(live, return_counts=True))}
    sk = np.array(skews)
    out["start_gap_us_percentiles"] = {q: round(float(np.percentile(sk, q)), 2) for q in (10, 25, 50, 75, 90)}
    one = keys[0]
    idx = np.where(cu == one)[0]
    o = np.argsort(start[idx])[:12]
    t00 = start[idx].min()
    out["cu0_timeline_us"] = [[round((start[idx][i] - t00) / 100.0, 1), round((end[idx][i] - t00) / 100.0, 1)]
                              for i in o]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
