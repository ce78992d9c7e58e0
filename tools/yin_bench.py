"""YIN prosody microbenchmark: 56 x 30 s utterances at 48 kHz (the vocoder side's share of
the bench step), time per launch and a hash of the per-hop f0 (A/B builds: JANUS_LIB).

python tools/yin_bench.py
"""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from janus_amd.services.prosody import prosody_launch  # noqa: E402
from janus_amd.workload import synth_speech  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = 56
    utts = [synth_speech(100 + i, 30.0) for i in range(B)]
    lengths = [len(u) for u in utts]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
    pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(dev)
    for _ in range(2):
        r = prosody_launch(pcm, offs, lengths, 48000, 512)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        r = prosody_launch(pcm, offs, lengths, 48000, 512)
    e1.record()
    torch.cuda.synchronize()
    h = hashlib.sha256(r.f0.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"yin B={B} x 30 s: {e0.elapsed_time(e1) / 5:.3f} ms per call, f0 sha256 {h} "
          f"(lib {os.environ.get('JANUS_LIB', 'default')})", flush=True)


if __name__ == "__main__":
    main()
