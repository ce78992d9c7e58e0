"""Standalone vocoder forward timing per kernel family (whole GPU, the bench's 64 x 30 s
batch) for A/B builds: JANUS_LIB=<alt .so> python tools/vocoder_ab.py [--reps 3]
-> one JSON line: forward ms (median), per-family ms of the last rep."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from janus_amd.vocoder import VocoderEngine, emotion_id  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    args = ap.parse_args()
    eng = VocoderEngine()
    B, F = args.batch, 2584
    lat = eng.frontend([b"(relaxed) ab %d" % i for i in range(B)], [emotion_id("relaxed")] * B, F)
    eng.forward(lat)  # warm-up
    torch.cuda.synchronize()
    times = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eng.set_timing(True)
        e0.record()
        eng.forward(lat)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    fam = {str(k): round(v["ms"] / args.reps, 2) for k, v in eng.family_stats(reset=True).items()}
    times.sort()
    print(json.dumps({"lib": os.environ.get("JANUS_LIB", "default"), "forward_ms": round(times[len(times) // 2], 2),
                      "all_ms": [round(t, 2) for t in times],
                      "families": fam}))


if __name__ == "__main__":
    main()
