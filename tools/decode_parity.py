"""Free-running greedy decode parity: janus_whisper_decode_greedy vs the fp32 KV-cached
oracle (oracle.whisper.greedy_cached) on the SAME encoder output, at full length.

Prints one JSON line: per utterance the GPU / oracle token counts, whether the whole
sequence matches, the first divergence and the oracle's top-2 margin there, and whether
the MessagePack packet built from each transcript matches. Usage (GPU box):
  python tools/decode_parity.py [--model base.en] [--n 6] [--max-length 448]
  python tools/decode_parity.py --bench 32     # the bench's own rows through its decode
--bench N: the first N utterances of bench.py's config-4 workload (30 s, seeds 4000 + i,
weights seed 0) decoded exactly as the headline step decodes them — JanusPipeline.
step_staggered (two slot sets, 224 positions per call, the decoder's CU-masked stream) —
against the oracle on the same encoder output; adds the token-agreement rate (positions
before the first divergence / tokens) and the packets (oracle detokeniser + packer on
each side's tokens).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from janus_amd.whisper import CONFIGS, WhisperEngine, synthetic_weights  # noqa: E402
from janus_amd.workload import synth_speech  # noqa: E402
from oracle import packet as opk  # noqa: E402
from oracle import whisper as ow  # noqa: E402

SECONDS = [30.0, 17.0, 8.0, 3.0, 1.0, 0.3, 24.0, 12.0]


def compare(eng, W, cfg, enc, max_length):
    tokens, ntok, slp = eng.decode(enc, max_length=max_length)
    torch.cuda.synchronize()
    tk = eng.tokenizer
    plen = len(tk.sot_sequence)
    toks, nt = tokens.cpu().numpy(), ntok.cpu().numpy()
    t0 = time.time()
    ref = ow.greedy_cached(enc.float().cpu(), W, cfg, tk, max_length)
    t_oracle = time.time() - t0
    rows = []
    tags = {"energy": "Normal", "pitch": "High"}
    for b in range(enc.shape[0]):
        g = [int(t) for t in toks[b][plen:plen + int(nt[b])]]
        r = ref[b]["tokens"]
        first = next((i for i in range(min(len(g), len(r))) if g[i] != r[i]),
                     None if len(g) == len(r) else min(len(g), len(r)))
        pk_g = opk.serialize(tk.transcript(g), 0, tags, "auto", 1.0)
        pk_r = opk.serialize(tk.transcript(r), 0, tags, "auto", 1.0)
        rows.append(dict(gpu_len=len(g), ref_len=len(r), match=g == r, first_diff=first,
                         margin_at_diff=(ref[b]["margins"][first] if first is not None and
                                         first < len(ref[b]["margins"]) else None),
                         min_margin=float(min(ref[b]["margins"])) if ref[b]["margins"] else None,
                         packet_match=pk_g == pk_r))
    return rows, t_oracle


def bench_rows(n, max_length):
    """--bench: the headline step's decode of the bench's first n utterances vs the oracle."""
    from janus_amd.pipeline import JanusPipeline
    cfg = CONFIGS["base.en"]
    W = synthetic_weights(cfg, 0)
    pipe = JanusPipeline("base.en", max_length=max_length, temperatures=(0.0,))
    dev = pipe.device
    utts = [synth_speech(4000 + i, 30.0) for i in range(n)]
    lengths = [len(u) for u in utts]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
    pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(dev)
    frames = 64
    outs = []
    for _ in range(2):   # the same batch twice: the second batch enters beside the first
        r = pipe.step_staggered(pcm, offs, lengths, frames)
        if r[0] is not None:
            outs.append(r[0])
    outs += [r[0] for r in pipe.flush_staggered(frames)]
    res = outs[0]
    w = pipe.whisper
    enc = w.encode(w.logmel(pcm, offs, n, 3))
    tk = w.tokenizer
    plen = len(tk.sot_sequence)
    toks, nt = res.tokens.cpu().numpy(), res.n_tokens.cpu().numpy()
    t0 = time.time()
    ref = ow.greedy_cached(enc.float().cpu(), W, cfg, tk, max_length)
    t_oracle = time.time() - t0
    tags = {"energy": "Normal", "pitch": "High"}
    rows = []
    agree = total = 0
    for b in range(n):
        g = [int(t) for t in toks[b][plen:plen + int(nt[b])]]
        r = ref[b]["tokens"]
        first = next((i for i in range(min(len(g), len(r))) if g[i] != r[i]),
                     None if len(g) == len(r) else min(len(g), len(r)))
        agree += len(r) if first is None else first
        total += len(r)
        rows.append(dict(gpu_len=len(g), ref_len=len(r), match=g == r, first_diff=first,
                         margin_at_diff=(ref[b]["margins"][first] if first is not None and
                                         first < len(ref[b]["margins"]) else None),
                         min_margin=float(min(ref[b]["margins"])) if ref[b]["margins"] else None,
                         packet_match=opk.serialize(tk.transcript(g), 0, tags, "auto", 1.0) ==
                         opk.serialize(tk.transcript(r), 0, tags, "auto", 1.0),
                         # the transcript the pipeline packed is the GPU tokens' transcript
                         text_is_tokens=res.texts[b] == tk.transcript(g)))
    same_twice = all(np.array_equal(outs[0].tokens.cpu().numpy(), o.tokens.cpu().numpy()) for o in outs[1:])
    margins = [r["margin_at_diff"] for r in rows if r["margin_at_diff"] is not None]
    return dict(model="base.en", n=n, max_length=max_length, path="JanusPipeline.step_staggered",
                oracle_s=round(t_oracle, 1),
                seq_match_rate=float(np.mean([r["match"] for r in rows])),
                packet_match_rate=float(np.mean([r["packet_match"] for r in rows])),
                token_agreement_rate=agree / max(total, 1),
                first_divergence_margins=margins,
                max_margin_at_divergence=max(margins) if margins else None,
                batches_identical=bool(same_twice), rows=rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench", type=int, default=0,
                    help="N > 0: the bench's first N utterances through the headline step")
    ap.add_argument("--model", default="base.en")
    ap.add_argument("--n", type=int, default=6)
    ap.add_argument("--max-length", type=int, default=448)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--e2e", action="store_true", help="also oracle front end + encoder")
    a = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    if a.bench > 0:
        print(json.dumps(bench_rows(a.bench, a.max_length)), flush=True)
        return
    cfg = CONFIGS[a.model]
    W = synthetic_weights(cfg, a.seed)
    eng = WhisperEngine(cfg, W)
    dev = eng.device
    utts = [synth_speech(140 + k, SECONDS[k % len(SECONDS)]) for k in range(a.n)]
    lengths = [len(u) for u in utts]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
    pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(dev)
    enc = eng.encode(eng.logmel(pcm, offs, len(utts), 3))
    rows, t_oracle = compare(eng, W, cfg, enc, a.max_length)
    out = dict(model=a.model, n=a.n, max_length=a.max_length, oracle_s=round(t_oracle, 1),
               seq_match_rate=float(np.mean([r["match"] for r in rows])),
               packet_match_rate=float(np.mean([r["packet_match"] for r in rows])), rows=rows)
    if a.e2e:
        # the oracle's own front end + fp32 encoder (output stored fp16, as the engine
        # hands it to the decoder), then the oracle decoder, vs the GPU's tokens
        from janus_amd.whisper import mel_filters
        t0 = time.time()
        mels = np.stack([ow.logmel(u, 3, mel_filters()) for u in utts])
        enc_ref = torch.cat([ow.encoder(mels[i:i + 2], W, cfg) for i in range(0, len(utts), 2)])
        enc_err = float((enc.float().cpu() - enc_ref).norm() / enc_ref.norm())
        ref = ow.greedy_cached(enc_ref.half().float(), W, cfg, eng.tokenizer, a.max_length)
        tokens, ntok, _ = eng.decode(enc, max_length=a.max_length)
        toks, nt = tokens.cpu().numpy(), ntok.cpu().numpy()
        plen = len(eng.tokenizer.sot_sequence)
        e2e = []
        for b in range(len(utts)):
            g = [int(t) for t in toks[b][plen:plen + int(nt[b])]]
            r = ref[b]["tokens"]
            first = next((i for i in range(min(len(g), len(r))) if g[i] != r[i]), None)
            e2e.append(dict(match=g == r, first_diff=first,
                            margin_at_diff=ref[b]["margins"][first] if first is not None else None))
        out["e2e"] = dict(enc_rel_err=enc_err, seconds=round(time.time() - t0, 1),
                          seq_match_rate=float(np.mean([r["match"] for r in e2e])), rows=e2e)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
