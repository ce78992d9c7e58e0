"""BASELINE config 5 on one GPU: S concurrent 48 kHz capture channels (default 16 = 128
channels / 8 GPUs) arriving in real time as 320 ms blocks (10 x 1536-sample chunks); per
block the speech gate runs for every chunk and phrases are segmented per channel
(engine.py:438-506). Completed phrases are encoded as one GPU batch (Whisper + YIN with
per-channel detector state + packet) and, in duplex mode, the packets are rendered by the
receiver leg (engine.py:220-286: prompt -> vocoder at the phrase's duration).

--async 1 (default): the encode + render runs on a worker stream while the next blocks
are ingested (StreamingEncoder(asynchronous=True)); --async 0: push blocks on it.
Prints one JSON line: per-block push latency p50 / p99, per-phrase duplex latency (phrase
completion -> packet + rendered audio) p50 / p99, the worker's deepest queue, and whether
both stay under the 320 ms block.

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
    ap.add_argument("--async", dest="asyn", type=int, default=1)
    ap.add_argument("--duplex", type=int, default=1)
    ap.add_argument("--fallback", action="store_true",
                    help="faster-whisper's temperature fallback on failing windows (the library "
                         "default); off by default here: seeded synthetic weights fail every window")
    a = ap.parse_args()
    import time
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
    from janus_amd.services.transcriber import TEMPERATURES
    temps = TEMPERATURES if a.fallback else (0.0,)
    rx = None
    if a.duplex:
        from janus_amd.pipeline import JanusPipeline
        rx = JanusPipeline(a.model, max_length=8)   # its vocoder renders the far end
    enc = StreamingEncoder(a.streams, w, max_length=a.max_length, asynchronous=bool(a.asyn),
                           receiver=rx, temperatures=temps)
    # warm-up: one block of silence + one short phrase batch (graph capture, allocations)
    warm = StreamingEncoder(a.streams, w, max_length=a.max_length, receiver=rx, temperatures=temps)
    z = np.zeros((a.streams, per_block * CHUNK), np.float32)
    sp = np.tile(synth_speech(1, per_block * CHUNK / 48000.0)[None, :per_block * CHUNK], (a.streams, 1))
    warm.push(sp)
    for _ in range(3):
        warm.push(z)
    torch.cuda.synchronize()
    phrases = 0
    t_start = time.perf_counter()
    for b in range(n_blocks):
        # blocks arrive in real time: block b is complete at t_start + (b + 1) * block
        wait = t_start + (b + 1) * a.block_ms / 1000.0 - time.perf_counter()
        if wait > 0:
            time.sleep(wait)
        out = enc.push(audio[:, b * per_block * CHUNK:(b + 1) * per_block * CHUNK])
        phrases += len(out)
    phrases += len(enc.flush())
    t_total = time.perf_counter() - t_start
    enc.close()
    lat = np.array(enc.latencies) * 1000.0
    plat = np.array(enc.phrase_latencies) * 1000.0 if enc.phrase_latencies else np.zeros(1)
    res = {"metric": "streaming latency (config 5)", "streams_per_gpu": a.streams,
           "block_ms": a.block_ms, "blocks": n_blocks, "phrases": phrases,
           "asynchronous": bool(a.asyn), "duplex": bool(a.duplex),
           "p50_ms": round(float(np.percentile(lat, 50)), 2),
           "p99_ms": round(float(np.percentile(lat, 99)), 2),
           "max_ms": round(float(lat.max()), 2),
           "phrase_p50_ms": round(float(np.percentile(plat, 50)), 2),
           "phrase_p99_ms": round(float(np.percentile(plat, 99)), 2),
           "phrase_max_ms": round(float(plat.max()), 2),
           "worker_max_queue": enc.max_queue,
           "wall_s": round(t_total, 2), "audio_s": round(n_blocks * a.block_ms / 1000.0, 2),
           "realtime": bool(np.percentile(lat, 99) < a.block_ms and np.percentile(plat, 99) < a.block_ms),
           "model": a.model, "max_length": a.max_length, "fallback": bool(a.fallback),
           "extra_seek_windows": enc.extra_windows,
           "data": "synthetic seeded speech phrases with silences; energy speech gate; seeded synthetic weights"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
