"""Kernel microbenchmarks (GPU): the vocoder's conv shapes through the kernel ABI.

python tools/kbench.py [--batch 16] [--reps 5]   -> one line per shape: ms, TFLOP/s, GB/s
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from janus_amd import _native as nat  # noqa: E402

# (name, Cin, Cout, taps, stride, pad, dil, transposed, pre, post, res, T_in per utt)
SHAPES = [
    ("pre512", 512, 512, 13, 1, 6, 1, 0, 0, 0, 0, 2584),
    ("up0", 512, 256, 0, 8, 4, 1, 1, 1, 0, 0, 2584),
    ("rb0_k3", 256, 256, 3, 1, 1, 1, 0, 1, 1, 0, 20672),
    ("rb0_k11d5", 256, 256, 11, 1, 25, 5, 0, 1, 1, 0, 20672),
    ("up1", 256, 128, 0, 8, 4, 1, 1, 1, 0, 0, 20672),
    ("rb1_k7d3", 128, 128, 7, 1, 9, 3, 0, 1, 1, 0, 165376),
    ("rb1_k7c2", 128, 128, 7, 1, 3, 1, 0, 0, 0, 1, 165376),
    ("rb2_k7d3", 64, 64, 7, 1, 9, 3, 0, 1, 1, 0, 330752),
    ("rb3_k7d3", 32, 32, 7, 1, 9, 3, 0, 1, 1, 0, 661504),
    ("rb4_k7d3", 16, 16, 7, 1, 9, 3, 0, 1, 1, 0, 1323008),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--units-only", action="store_true")
    ap.add_argument("--xattn", action="store_true")
    ap.add_argument("--wide", action="store_true")
    ap.add_argument("--dec", action="store_true")
    ap.add_argument("--lngemm", action="store_true")
    a = ap.parse_args()
    if a.lngemm:
        lngemm_bench()
        return
    if a.dec:
        dec_bench()
        return
    if a.xattn:
        xattn_bench()
        return
    if a.wide:
        wide_units(a.batch, a.reps)
        return
    if a.units_only:
        resunits(a.batch, a.reps)
        return
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    B = a.batch
    if not a.only:
        resunits(B, a.reps)
    for (name, Cin, Cout, taps, stride, pad, dil, tr, pre, post, use_res, T_in) in SHAPES:
        if a.only and a.only not in name:
            continue
        if tr:
            T_out = T_in * stride
            real_taps = 2
        else:
            T_out = (T_in + 2 * pad - dil * (taps - 1) - 1) // stride + 1
            real_taps = taps
        x = torch.randn(B, T_in, Cin, device=dev).half()
        wshape = (Cin, Cout, 2 * stride) if tr else (Cout, Cin, taps)
        w = (torch.randn(*wshape, device=dev) / math.sqrt(Cin * real_taps)).float()
        bias = torch.randn(Cout, device=dev) * 0.1
        n = nat.lib().janus_conv1d_packed_size(Cin, Cout, taps, tr, stride)
        packed = torch.empty(n, dtype=torch.float16, device=dev)
        nat.call("janus_conv1d_pack", w.data_ptr(), packed.data_ptr(), Cin, Cout, taps, tr, stride, s)
        out = torch.empty(B, T_out, Cout, device=dev, dtype=torch.float16)
        res = torch.randn(B, T_out, Cout, device=dev).half() if use_res else None

        def run():
            nat.call("janus_conv1d_f16", x.data_ptr(), B, T_in, Cin, packed.data_ptr(), bias.data_ptr(),
                     out.data_ptr(), T_out, Cout, taps, stride, pad, dil, tr, pre, post,
                     res.data_ptr() if res is not None else None, T_out * Cout, 1.0, 0, s)

        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        flops = 2.0 * Cin * Cout * real_taps * T_out * B
        byts = 2.0 * B * (T_in * Cin + T_out * Cout * (2 if use_res else 1))
        print(f"{name:10s} B={B} T_out={T_out:8d} {ms:8.3f} ms {flops / ms / 1e9:8.1f} TF/s "
              f"{byts / ms / 1e6:8.1f} GB/s", flush=True)


def resunits(B, reps):
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    for (C, k, d, T) in [(32, 7, 3, 661504), (32, 11, 5, 661504), (16, 7, 3, 1323008), (16, 3, 1, 1323008)]:
        x = torch.randn(B, T, C, device=dev).half()
        out = torch.empty_like(x)
        n = nat.lib().janus_resunit_packed_size(C, k)
        w = (torch.randn(C, C, k, device=dev) / math.sqrt(C * k)).float()
        p = torch.empty(n, dtype=torch.float16, device=dev)
        nat.call("janus_resunit_pack", w.data_ptr(), p.data_ptr(), C, k, s)
        bias = torch.zeros(C, device=dev)

        def run():
            nat.call("janus_resunit_f16", x.data_ptr(), out.data_ptr(), p.data_ptr(), bias.data_ptr(),
                     p.data_ptr(), bias.data_ptr(), B, T, C, k, d, 1.0 / 3.0, 1, s)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        flops = 2 * 2.0 * C * C * k * T * B
        byts = 2.0 * B * T * C * 3  # read x, read+write the ParallelBlock accumulator
        print(f"unit C{C} k{k} d{d} B={B} T={T:8d} {ms:8.3f} ms {flops / ms / 1e9:8.1f} TF/s "
              f"{byts / ms / 1e6:8.1f} GB/s", flush=True)




def _time(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def wide_units(B, reps):
    """Fused ResBlock1 unit (resunit_wide.hip) vs the same unit as two conv launches."""
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    shapes = [(256, 3, 1, 20672), (256, 11, 5, 20672), (128, 3, 1, 165376), (128, 7, 3, 165376),
              (128, 11, 5, 165376), (64, 3, 1, 330752), (64, 7, 3, 330752), (64, 11, 5, 330752)]
    if os.environ.get("WIDE_C"):  # every (k, d) of one channel count
        C = int(os.environ["WIDE_C"])
        T = {256: 20672, 128: 165376, 64: 330752}[C]
        shapes = [(C, k, d, T) for k in (3, 7, 11) for d in (1, 3, 5)]
    for (C, k, d, T) in shapes:
        x = torch.randn(B, T, C, device=dev).half()
        out = torch.empty_like(x)
        mid = torch.empty_like(x)
        w = [(torch.randn(C, C, k, device=dev) / math.sqrt(C * k)).float() for _ in range(2)]
        bias = torch.zeros(C, device=dev)
        n = nat.lib().janus_resunit_packed_size(C, k)
        pu = [torch.empty(n, dtype=torch.float16, device=dev) for _ in range(2)]
        pc = [torch.empty(nat.lib().janus_conv1d_packed_size(C, C, k, 0, 1), dtype=torch.float16, device=dev)
              for _ in range(2)]
        for i in range(2):
            nat.call("janus_resunit_pack", w[i].data_ptr(), pu[i].data_ptr(), C, k, s)
            nat.call("janus_conv1d_pack", w[i].data_ptr(), pc[i].data_ptr(), C, C, k, 0, 1, s)

        def fused():
            nat.call("janus_resunit_f16", x.data_ptr(), out.data_ptr(), pu[0].data_ptr(), bias.data_ptr(),
                     pu[1].data_ptr(), bias.data_ptr(), B, T, C, k, d, 1.0 / 3.0, 1, s)

        def pair():
            nat.call("janus_conv1d_f16", x.data_ptr(), B, T, C, pc[0].data_ptr(), bias.data_ptr(),
                     mid.data_ptr(), T, C, k, 1, d * (k - 1) // 2, d, 0, 1, 1, None, 0, 1.0, 0, s)
            nat.call("janus_conv1d_f16", mid.data_ptr(), B, T, C, pc[1].data_ptr(), bias.data_ptr(),
                     out.data_ptr(), T, C, k, 1, (k - 1) // 2, 1, 0, 0, 0, x.data_ptr(), T * C,
                     1.0 / 3.0, 1, s)
        flops = 2 * 2.0 * C * C * k * T * B
        mf, mp = _time(fused, reps), _time(pair, reps)
        print(f"wide C{C:3d} k{k:2d} d{d} B={B} T={T:7d} fused {mf:7.3f} ms {flops / mf / 1e9:7.1f} TF/s | "
              f"two convs {mp:7.3f} ms {flops / mp / 1e9:7.1f} TF/s", flush=True)


def _time_cold(fn, reps, flush):
    """Mean time of fn with the caches flushed (a 512 MB write) before every call."""
    fn()
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(reps):
        if flush is not None:
            flush.fill_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        tot += e0.elapsed_time(e1)
    return tot / reps


def xattn_bench(reps=20):
    """Absorbed cross-attention at the bench shape (64 x 1500 x 512, 8 heads) per split
    count, caches flushed before every call (the decoder reads enc once per layer)."""
    dev = torch.device("cuda", 0)
    if os.environ.get("XMASK"):  # on a CU-masked stream: XMASK CUs per XCD (the decoder's share)
        n = torch.cuda.get_device_properties(0).multi_processor_count
        ms = nat.MaskedStream(nat.split_cu_masks(n, int(os.environ["XMASK"]))[0])
        torch.cuda.set_stream(ms.stream)
        print(f"masked stream: {ms.n_cus} CUs", flush=True)
    s = torch.cuda.current_stream().cuda_stream
    B, Te, D, H = 64, 1500, 512, 8
    enc = torch.randn(B, Te, D, device=dev).half()
    qk = (torch.randn(B, H, D, device=dev) * 0.1).half()
    out = torch.empty(B, H * D, device=dev, dtype=torch.float16)
    flush = torch.empty(128 << 20, device=dev)
    for ns in [int(v) for v in os.environ.get("XSPLITS", "1,2,4,8,12,16,24").split(",")]:
        pc = torch.empty(B * ns * H * D, device=dev)
        pml = torch.empty(B * ns * H * 2, device=dev)

        def run():
            nat.call("janus_cross_attention_f16", qk.data_ptr(), enc.data_ptr(), B, Te, D, H, ns,
                     pc.data_ptr(), pml.data_ptr(), out.data_ptr(), s)
        ms = _time_cold(run, reps, flush)
        print(f"xattn nsplit={ns:3d} {ms * 1000:8.1f} us  {B * Te * D * 2 / ms / 1e6:8.1f} GB/s (enc, cold)",
              flush=True)
        ms = _time_cold(run, reps, None)
        print(f"xattn nsplit={ns:3d} {ms * 1000:8.1f} us  {B * Te * D * 2 / ms / 1e6:8.1f} GB/s (enc, warm)",
              flush=True)


def dec_bench(reps=20):
    """Decoder self-attention (64 utterances, 8 heads, cache [64][448][512]) per cache length."""
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    B, H, NC = 64, 8, 448
    d = H * 64
    q = torch.randn(B, 3 * d, device=dev).half()
    k = torch.randn(B, NC, d, device=dev).half()
    v = torch.randn(B, NC, d, device=dev).half()
    out = torch.empty(B, d, device=dev, dtype=torch.float16)
    po = torch.empty(B * 8 * d, device=dev)
    pm = torch.empty(B * 8 * H * 2, device=dev)
    flush = torch.empty(128 << 20, device=dev)
    for T in (16, 64, 224, 448):
        def run():
            nat.call("janus_decode_attention_f16", q.data_ptr(), 3 * d, k.data_ptr(), v.data_ptr(),
                     NC * d, d, T, out.data_ptr(), d, B, H, 0.125, po.data_ptr(), pm.data_ptr(), s)
        ms = _time_cold(run, reps, flush)
        print(f"self-attn T={T:4d} {ms * 1000:8.1f} us  {B * T * d * 4 / ms / 1e6:8.1f} GB/s (K+V, cold)",
              flush=True)


def lngemm_bench(reps=50):
    """Decoder pre-LN projection, M = 64, K = 512: LayerNorm launch + skinny GEMM vs the GEMM
    with the LayerNorm in its prologue; warm (back to back) and with x rewritten by a kernel
    just before (as the residual GEMM does in the decoder)."""
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    M, K = 64, 512
    x = torch.randn(M, K, device=dev)
    g = torch.ones(K, device=dev)
    b = torch.zeros(K, device=dev)
    a = torch.empty(M, K, device=dev, dtype=torch.float16)
    for N in (1536, 2048, 4096):
        W = (torch.randn(N, K, device=dev) * 0.04).half()
        out = torch.empty(M, N, device=dev, dtype=torch.float16)

        def sep():
            nat.call("janus_layernorm_f16", x.data_ptr(), g.data_ptr(), b.data_ptr(), a.data_ptr(), M, K,
                     1e-5, s)
            nat.call("janus_gemm_f16", 0, a.data_ptr(), K, W.data_ptr(), K, None, out.data_ptr(), N, None, 0,
                     M, N, K, s)

        def fused():
            nat.call("janus_gemm_ln_f16", 0, x.data_ptr(), K, g.data_ptr(), b.data_ptr(), 1e-5, W.data_ptr(),
                     K, None, out.data_ptr(), N, M, N, K, s)

        def touch(fn):
            def run():
                x.add_(0.0)
                fn()
            return run
        t = [_time(f, reps) * 1000 for f in (sep, fused, touch(sep), touch(fused))]
        tx = _time(lambda: x.add_(0.0), reps) * 1000
        print(f"N={N:5d} LN+GEMM {t[0]:6.1f} us  fused {t[1]:6.1f} us | after a write of x: "
              f"LN+GEMM {t[2] - tx:6.1f} us  fused {t[3] - tx:6.1f} us (write {tx:.1f} us)", flush=True)


if __name__ == "__main__":
    main()
