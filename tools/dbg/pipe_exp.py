"""Experiment: encode(batch i) overlapped with decode(batch i-1) on a second stream."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from janus_amd.pipeline import JanusPipeline  # noqa: E402
from janus_amd.workload import synth_speech  # noqa: E402

K = int(os.environ.get("K", "4"))
dev = torch.device("cuda", 0)
utts = [synth_speech(4000 + i, 30.0) for i in range(64)]
lengths = [len(u) for u in utts]
offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(dev)
frames = 2584
pipe = JanusPipeline("base.en", max_length=448)
pipe.step(pcm, offs, lengths, frames)
torch.cuda.synchronize()

t0 = time.perf_counter()
for _ in range(K):
    pipe.step(pcm, offs, lengths, frames)
torch.cuda.synchronize()
seq = (time.perf_counter() - t0) / K

prio = int(os.environ.get("VPRIO", "0"))
vs = torch.cuda.Stream(device=dev, priority=prio)
main = torch.cuda.current_stream(dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
prev = None
for i in range(K + 1):
    if prev is not None:
        vs.wait_stream(main)
        with torch.cuda.stream(vs):
            pipe.decode(prev.packets, frames)
    if i < K:
        prev = pipe.encode(pcm, offs, lengths)
torch.cuda.synchronize()
ovl = (time.perf_counter() - t0) / K
print(f"sequential {seq * 1000:.1f} ms/step   overlapped {ovl * 1000:.1f} ms/step (K={K}, vprio={prio})", flush=True)
