"""Log-mel front end microbenchmark: 64 x 30 s utterances at 48 kHz (decimated to 16 kHz,
the bench workload), time per launch and a hash of the output (A/B builds: JANUS_LIB).

python tools/mel_bench.py
"""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from janus_amd.whisper import CONFIGS, WhisperEngine, synthetic_weights  # noqa: E402
from janus_amd.workload import synth_speech  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cfg = CONFIGS["tiny.en"]  # the front end does not depend on the model size
    eng = WhisperEngine(cfg, synthetic_weights(cfg, seed=5))
    B = 64
    utts = [synth_speech(100 + i, 30.0) for i in range(B)]
    lengths = [len(u) for u in utts]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
    pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(dev)
    for _ in range(3):
        mel = eng.logmel(pcm, offs, B, 3)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        mel = eng.logmel(pcm, offs, B, 3)
    e1.record()
    torch.cuda.synchronize()
    h = hashlib.sha256(mel.contiguous().cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"logmel B={B} x 30 s: {e0.elapsed_time(e1) / 20:.3f} ms per call, sha256 {h} "
          f"(lib {os.environ.get('JANUS_LIB', 'default')})", flush=True)


if __name__ == "__main__":
    main()
