"""BASELINE config 5 on one GPU: S concurrent 48 kHz capture channels (default 16 = 128
channels / 8 GPUs) advanced in 320 ms blocks (10 x 1536-sample chunks); per block the
speech gate runs for every chunk, phrases are segmented per channel (engine.py:438-506)
and every phrase completed in that block is encoded as one GPU batch (Whisper + YIN with
per-channel detector state + packet). Prints one JSON line: per-block latency p50 / p99
(ms), phrases, and whether p50 stays under the 320 ms block (real time).

python tools/stream_bench.py [--streams 16] [--seconds 30] [--model base.en] [--max-length 448]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--model", default="base.en")
    ap.add_argument("--max-length", type=int, default=448)
    ap.add_argument("--block-ms", type=int, default=320)
    a = ap.parse_args()
    import torch
    from janus_amd.streaming import CHUNK, StreamingEncoder
    from janus_amd.whisper import CONFIGS, WhisperEngine
    from janus_amd.workload import synth_speech
    per_block = int(round(a.block_ms / 32.0))          # 1536 samples = 32 ms
    n_blocks = int(a.seconds * 1000 / a.block_ms)
    total = n_blocks * per_block * CHUNK
    rng = np.random.default_rng(5000)
    audio = np.zeros((a.streams, total), np.float32)
    for s in range(a.streams):  # phrases of 1.5-6 s separated by 0.6-2 s of silence
        t = int(rng.integers(0, 48000))
        k = 0
        while t < total:
            ph = synth_speech(5000 + 97 * s + k, float(rng.uniform(1.5, 6.0)))
            n = min(len(ph), total - t)
            audio[s, t:t + n] = ph[:n]
            t += n + int(rng.uniform(0.6, 2.0) * 48000)
            k += 1
    w = WhisperEngine(CONFIGS[a.model], seed=0)
    enc = StreamingEncoder(a.streams, w, max_length=a.max_length)
    # warm-up: one block of silence + one short phrase batch (graph capture, allocations)
    warm = StreamingEncoder(a.streams, w, max_length=a.max_length)
    z = np.zeros((a.streams, per_block * CHUNK), np.float32)
    sp = np.tile(synth_speech(1, per_block * CHUNK / 48000.0)[None, :per_block * CHUNK], (a.streams, 1))
    warm.push(sp)
    for _ in range(3):
        warm.push(z)
    torch.cuda.synchronize()
    phrases = 0
    for b in range(n_blocks):
        out = enc.push(audio[:, b * per_block * CHUNK:(b + 1) * per_block * CHUNK])
        phrases += len(out)
    lat = np.array(enc.latencies) * 1000.0
    res = {"metric": "streaming per-block latency (config 5)", "streams_per_gpu": a.streams,
           "block_ms": a.block_ms, "blocks": n_blocks, "phrases": phrases,
           "p50_ms": round(float(np.percentile(lat, 50)), 2),
           "p99_ms": round(float(np.percentile(lat, 99)), 2),
           "max_ms": round(float(lat.max()), 2),
           "mean_ms": round(float(lat.mean()), 2),
           "realtime_p50": bool(np.percentile(lat, 50) < a.block_ms),
           "model": a.model, "max_length": a.max_length,
           "data": "synthetic seeded speech phrases with silences; energy speech gate; seeded synthetic weights"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
