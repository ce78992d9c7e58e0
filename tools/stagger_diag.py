"""Where does a staggered decode first differ from the full one? (diagnostic, GPU)
Mirrors tests/test_whisper_gpu.py::test_staggered_decode_matches_full, printing per batch
and row the first differing token and the summed log-probabilities; the full decodes run
before and after the staggered calls."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from janus_amd.whisper import CONFIGS, DecodeOut, WhisperEngine, synthetic_weights
    from janus_amd.workload import synth_speech
    cfg = CONFIGS["tiny.en"]
    eng = WhisperEngine(cfg, synthetic_weights(cfg, seed=5))
    dev = torch.device("cuda", 0)
    N = 3

    def pack(utts):
        lengths = [len(u) for u in utts]
        offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
        pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(dev)
        return pcm, offs

    def cmp(tag, a, b):
        ta, tb = a.tokens.cpu(), b.tokens.cpu()
        for j in range(N):
            d = (ta[j] != tb[j]).nonzero()
            first = int(d[0]) if len(d) else None
            print(f"{tag} row {j}: first token diff {first}, sum_lp {float(a.sum_logprob[j]):.4f} vs "
                  f"{float(b.sum_logprob[j]):.4f}", flush=True)

    for L in (40, 448):
        S = L // 2
        batches = []
        for k in range(3):
            pcm, offs = pack([synth_speech(300 + 10 * k + j, 1.5 + j) for j in range(N)])
            batches.append(eng.encode(eng.logmel(pcm, offs, N, 3)))
        ref = [eng.decode_ex(e, max_length=L) for e in batches]
        sets, got = [None, None], {}
        for call in range(4):
            fresh, cont = call % 2, 1 - call % 2
            sets[fresh] = call if call < 3 else None
            rows_enc, offs = [], []
            for st in (0, 1):
                bi = sets[st]
                if bi is None:
                    rows_enc.append(torch.zeros_like(batches[0]))
                    offs += [L - S] * N if st == cont or call == 3 else [0] * N
                else:
                    rows_enc.append(batches[bi])
                    offs += [0 if st == fresh else S] * N
            if call == 0:
                offs = [0] * (2 * N)
            out = eng.decode_ex(torch.cat(rows_enc), max_length=L, pos_offset=offs, steps=S)
            print(f"L={L} call {call}: offsets {offs}", flush=True)
            if call > 0 and sets[cont] is not None:
                bi = sets[cont]
                sl = slice(cont * N, cont * N + N)
                got[bi] = DecodeOut(out.tokens[sl].clone(), out.n_tokens[sl].clone(),
                                    out.sum_logprob[sl].clone(), out.no_speech_prob[sl].clone(),
                                    out.prompt_lens[sl])
                sets[cont] = None
        ref2 = [eng.decode_ex(e, max_length=L) for e in batches]
        for bi in range(3):
            cmp(f"L={L} batch {bi} ref vs ref-after", ref[bi], ref2[bi])
            cmp(f"L={L} batch {bi} ref vs staggered", ref[bi], got[bi])


if __name__ == "__main__":
    main()
