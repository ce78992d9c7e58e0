"""Locate resunit parity errors by row (debug helper)."""
import math, sys, os
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from janus_amd import _native as nat

def run(C, k, d, acc, T, B=2):
    gpu = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(C * 100 + k * 10 + d)
    x = torch.randn(B, T, C, generator=g).half()
    w1 = torch.randn(C, C, k, generator=g) / math.sqrt(C * k)
    w2 = torch.randn(C, C, k, generator=g) / math.sqrt(C * k)
    b1 = torch.randn(C, generator=g) * 0.1
    b2 = torch.randn(C, generator=g) * 0.1
    prev = torch.randn(B, T, C, generator=g).half()
    scale = 1 / 3 if acc else 1.0
    xd = x.double().transpose(1, 2)
    h = F.conv1d(F.silu(xd).half().double(), w1.half().double(), b1.double(), padding=d * (k - 1) // 2, dilation=d)
    h = F.silu(h).half().double()
    y = F.conv1d(h, w2.half().double(), b2.double(), padding=(k - 1) // 2) + xd
    ref = y.transpose(1, 2) * scale + (prev.double() if acc else 0)
    n = nat.lib().janus_resunit_packed_size(C, k)
    p1 = torch.empty(n, dtype=torch.float16, device=gpu); p2 = torch.empty_like(p1)
    dw1, dw2 = w1.to(gpu), w2.to(gpu)
    nat.call("janus_resunit_pack", dw1.data_ptr(), p1.data_ptr(), C, k, s)
    nat.call("janus_resunit_pack", dw2.data_ptr(), p2.data_ptr(), C, k, s)
    dx, db1, db2 = x.to(gpu), b1.to(gpu), b2.to(gpu)
    out = prev.to(gpu).clone()
    nat.call("janus_resunit_f16", dx.data_ptr(), out.data_ptr(), p1.data_ptr(), db1.data_ptr(),
             p2.data_ptr(), db2.data_ptr(), B, T, C, k, d, scale, acc, s)
    torch.cuda.synchronize()
    e = (out.double().cpu() - ref).abs().amax(dim=2)  # [B][T]
    bad = (e > 0.02).nonzero()
    print(f"C{C} k{k} d{d} acc{acc} T{T}: max err {float(e.max()):.4f}, bad rows {len(bad)}")
    if len(bad):
        rows = bad[:, 1].tolist()
        print("  first bad (b,t):", bad[:20].tolist())
        print("  t mod 240 histogram:", sorted(set(r % 240 for r in rows))[:40])

for cfg in [(16, 11, 5, 1, 1500), (16, 11, 5, 0, 1500), (16, 7, 5, 1, 1500), (16, 11, 3, 1, 1500), (32, 11, 5, 1, 1500), (16, 3, 1, 0, 1500)]:
    run(*cfg)
