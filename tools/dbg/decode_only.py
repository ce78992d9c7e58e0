"""Greedy decode of 64 synthetic encoder outputs (base.en), for PMC passes over the
decoder kernels: python tools/dbg/decode_only.py [max_length]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from janus_amd.whisper import CONFIGS, WhisperEngine  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 64
w = WhisperEngine(CONFIGS["base.en"], seed=0)
g = torch.Generator(device="cuda").manual_seed(0)
enc = (torch.randn(64, 1500, 512, device="cuda", generator=g) * 0.5).half()
w.decode(enc, L)
torch.cuda.synchronize()
print("decoded", L)
