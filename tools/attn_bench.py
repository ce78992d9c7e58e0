"""Encoder attention microbenchmark: B=64, T=1500, H=8 (base.en), both kernel forms."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from janus_amd import _native as nat  # noqa: E402


def main():
    B, T, H = 64, 1500, 8
    d = H * 64
    dev = torch.device("cuda", 0)
    qkv = (torch.randn(B, T, 3 * d, device=dev) * 1.5).half()
    out = torch.empty(B, T, d, dtype=torch.float16, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    run = lambda: nat.call("janus_attention_f16", qkv.data_ptr(), out.data_ptr(), B, T, H, 0.125, s)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    fl = 4.0 * B * H * T * T * 64
    print(f"attention B={B} T={T} H={H}: {ms:.3f} ms {fl / ms / 1e9:.1f} TF/s "
          f"({'v1' if os.environ.get('JANUS_ATTN_V1') else 'st'})", flush=True)


if __name__ == "__main__":
    main()
