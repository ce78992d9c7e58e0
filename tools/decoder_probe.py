"""Decoder-side probe: the greedy decoder of the bench workload (64 x 30 s, base.en,
447 positions) on a CU-masked stream of `dec_per_xcd` CUs per XCD, alone and beside the
vocoder (batch 64 x 30 s on the complementary CUs), to separate the decoder's own latency
floor from interference. Prints one JSON line per configuration.

python tools/decoder_probe.py [--per-xcd 8,12,16,24] [--beside 1] [--rows 128] [--persistent 1]
(--rows 128: the headline step's two slot sets, the 64 encoder rows twice)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-xcd", default="8,12,16,24")
    ap.add_argument("--beside", type=int, default=1)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--max-length", type=int, default=448)
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--persistent", type=int, default=0)
    ap.add_argument("--xsplits", type=int, default=4)
    a = ap.parse_args()
    import numpy as np
    import torch
    from janus_amd import _native as nat
    from janus_amd.pipeline import JanusPipeline
    from janus_amd.workload import synth_speech
    dev = torch.device("cuda", 0)
    B = 64
    utts = [synth_speech(4000 + i, 30.0) for i in range(B)]
    offs = torch.tensor(np.concatenate([[0], np.cumsum([len(u) for u in utts])]), dtype=torch.int64, device=dev)
    pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(dev)
    pipe = JanusPipeline("base.en", max_length=448, temperatures=(0.0,))
    w = pipe.whisper
    enc = w.encode(w.logmel(pcm, offs, B, 3))
    if a.rows > B:
        enc = torch.cat([enc] * ((a.rows + B - 1) // B))[:a.rows].contiguous()
    frames = 2584
    lat = None
    if a.beside:
        lat = pipe.vocoder.frontend([b"(auto) probe text"] * B, [0] * B, frames)
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    for per in [int(x) for x in a.per_xcd.split(",")]:
        dmask, vmask = nat.split_cu_masks(n, per)
        ds, vs = nat.MaskedStream(dmask, dev), nat.MaskedStream(vmask, dev)
        for beside in ([0, 1] if a.beside else [0]):
            for rep in range(a.reps):
                torch.cuda.synchronize()
                e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                e[0].record(ds.stream)
                e[2].record(vs.stream)
                if beside:
                    with torch.cuda.stream(vs.stream):
                        pipe.vocoder.forward(lat, want_pcm=True)
                e[3].record(vs.stream)
                with torch.cuda.stream(ds.stream):
                    out = w.decode_ex(enc, max_length=a.max_length, xattn_splits=a.xsplits, cu_count=ds.n_cus,
                                      persistent=a.persistent)
                e[1].record(ds.stream)
                torch.cuda.synchronize()
                print(json.dumps({"dec_per_xcd": per, "beside_vocoder": beside, "rep": rep,
                                  "decoder_ms": round(e[0].elapsed_time(e[1]), 1),
                                  "vocoder_ms": round(e[2].elapsed_time(e[3]), 1) if beside else None,
                                  "tokens": int(out.n_tokens.float().mean().item()), "rows": int(enc.shape[0]),
                                  "persistent": a.persistent, "xsplits": a.xsplits}), flush=True)


if __name__ == "__main__":
    main()
