"""Config-5 phrase decode latency (one round of generate_segments on a few phrases, base.en,
max_length 448): the T = 0 rows alone and the speculative round (T = 0 row + 5 temperatures
x best_of 5 per window), on the launch path vs the persistent segments (which take no
shared encoder rows: the speculative round then replicates each window's encoder output per
row). Prints one JSON line per configuration (median ms of 5 calls).

python tools/stream_decode_probe.py [n_windows=2]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from janus_amd.services.transcriber import TEMPERATURES, fallback_seed
    from janus_amd.whisper import CONFIGS, WhisperEngine
    from janus_amd.workload import synth_speech
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda", 0)
    w = WhisperEngine(CONFIGS["base.en"], seed=0)
    utts = [synth_speech(700 + k, 3.0 + k) for k in range(n)]
    offs = torch.tensor(np.concatenate([[0], np.cumsum([len(u) for u in utts])]), dtype=torch.int64, device=dev)
    pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(dev)
    enc = w.encode(w.logmel(pcm, offs, n, 3))
    sot = list(w.tokenizer.sot_sequence)
    per = 1 + 5 * 5
    temps, seeds, eidx = [], [], []
    for j in range(n):
        temps.append(0.0)
        seeds.append(0)
        for ti in range(1, 6):
            temps += [float(TEMPERATURES[ti])] * 5
            seeds += [fallback_seed(j, 0, ti, h) for h in range(5)]
        eidx += [j] * per
    rep = enc.index_select(0, torch.tensor(eidx, device=dev)).contiguous()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1000.0)
        return round(float(np.median(ts)), 1)
    res = {"windows": n}
    for p in (0, 2):
        res[f"t0_persist{p}_ms"] = timed(lambda: w.decode_ex(enc, prompts=[sot] * n, max_length=448, persistent=p))
    res["spec_shared_launch_ms"] = timed(lambda: w.decode_ex(enc, prompts=[sot] * (n * per), max_length=448,
                                                             temperature=temps, seeds=seeds, enc_index=eidx))
    for p in (0, 2):
        res[f"spec_replicated_persist{p}_ms"] = timed(lambda: w.decode_ex(rep, prompts=[sot] * (n * per), max_length=448,
                                                                          temperature=temps, seeds=seeds, persistent=p))
    a = w.decode_ex(enc, prompts=[sot] * (n * per), max_length=448, temperature=temps, seeds=seeds, enc_index=eidx)
    b = w.decode_ex(rep, prompts=[sot] * (n * per), max_length=448, temperature=temps, seeds=seeds, persistent=2)
    res["replicated_persist_identical"] = bool(torch.equal(a.tokens.cpu(), b.tokens.cpu()) and
                                               torch.equal(a.sum_logprob.cpu(), b.sum_logprob.cpu()))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
