"""How faster-whisper's seek loop walks the bench's 30 s clips: runs the drop-in's batched
generate_segments (T = 0 by default) on the bench workload (seeds 4000 + i, 48 kHz, [::3])
and prints, per round, the active clips, their seeks and prompt lengths, plus the wall
time of each round and in total. One JSON line to stdout.

    python tools/seek_probe.py [--batch 64] [--model base.en] [--fallback]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--model", default="base.en")
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--fallback", action="store_true")
    a = ap.parse_args()
    from janus_amd.services import transcriber as tr
    from janus_amd.whisper import CONFIGS, WhisperEngine
    from janus_amd.workload import synth_speech
    w = WhisperEngine(CONFIGS[a.model], seed=0)
    auds = [np.ascontiguousarray(synth_speech(4000 + i, a.seconds)[::3]) for i in range(a.batch)]
    temps = tr.TEMPERATURES if a.fallback else (0.0,)
    # one warm pass (graph capture) on two clips
    tr.generate_segments(w, auds[:2], temperatures=(0.0,))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    streams = tr.generate_segments(w, auds, temperatures=temps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    wins = [s.windows for s in streams]
    out = {"batch": a.batch, "model": a.model, "fallback": a.fallback, "seconds_total": round(dt, 3),
           "windows_total": int(sum(wins)), "windows_hist": {int(k): int(v) for k, v in
                                                            zip(*np.unique(wins, return_counts=True))},
           "segments_total": int(sum(len(s.segments) for s in streams)),
           "seeks_first": [int(s.segments[0].seek) if s.segments else -1 for s in streams[:8]],
           "segment_seeks": [[int(g.seek) for g in s.segments][:12] for s in streams[:6]],
           "tokens_all": [len(s.all_tokens) for s in streams[:16]],
           "xrt_stt_only": round(a.batch * a.seconds / dt, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
