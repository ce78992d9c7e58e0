"""GPU parity of the kernel-level ABI (include/janus_kernels.h) against PyTorch fp32/fp64
CPU references of the same ops on the same fp16-rounded inputs."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from janus_amd import _native as nat

pytestmark = pytest.mark.gpu


def stream():
    return torch.cuda.current_stream().cuda_stream


def rel_err(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("M,N,K", [(300, 200, 64), (64, 1536, 512), (1, 24, 8), (1500, 512, 2048),
                                   (129, 130, 136), (64, 4096, 512), (20, 2056, 384), (7, 2304, 200)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemm(gpu, M, N, K, epi):
    g = torch.Generator().manual_seed(M * 7 + N + K + epi)
    A = (torch.randn(M, K, generator=g)).half()
    W = (torch.randn(N, K, generator=g) / math.sqrt(K)).half()
    bias = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    ref = A.double() @ W.double().T + bias.double()
    if epi == 1:
        ref = F.gelu(ref)
    if epi == 2:
        ref = ref + R.double()
    dA, dW, db = A.to(gpu), W.to(gpu), bias.to(gpu)
    out_dtype = torch.float16 if epi in (0, 1) else torch.float32
    C = R.to(gpu).clone() if epi == 2 else torch.empty(M, N, dtype=out_dtype, device=gpu)
    nat.call("janus_gemm_f16", epi, dA.data_ptr(), K, dW.data_ptr(), K, db.data_ptr(), C.data_ptr(),
             N, C.data_ptr() if epi == 2 else None, N, M, N, K, stream())
    torch.cuda.synchronize()
    err = rel_err(C, ref)
    assert err < (2e-3 if out_dtype == torch.float16 else 1e-4), err


@pytest.mark.parametrize("M,N,K", [(3000, 1536, 512), (256, 512, 512), (4500, 2048, 512),
                                   (3000, 512, 2048), (257, 256, 64), (300, 256, 128)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemm_big(gpu, M, N, K, epi):
    """The encoder-size kernel (janus_gemm_f16 with N % 256 == 0, K % 64 == 0 -> gemm_big:
    256 x 256 tiles, LDS-DMA staging) against an fp64 reference, ragged M included, and
    bit-identical to the 128 x 128-tile kernel (same k-step order per output)."""
    g = torch.Generator().manual_seed(M + N * 5 + K + epi)
    A = (torch.rand(M, K, generator=g) * 2 - 1).half()
    W = ((torch.rand(N, K, generator=g) * 2 - 1) / math.sqrt(K)).half()
    bias = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    ref = A.double() @ W.double().T + bias.double()
    if epi == 1:
        ref = F.gelu(ref)
    if epi == 2:
        ref = ref + R.double()
    dA, dW, db = A.to(gpu), W.to(gpu), bias.to(gpu)
    out_dtype = torch.float16 if epi in (0, 1) else torch.float32
    outs = []
    for fn in ("janus_gemm_f16", "janus_gemm_nt128_f16"):
        C = R.to(gpu).clone() if epi == 2 else torch.full((M, N), float("nan"), dtype=out_dtype, device=gpu)
        nat.call(fn, epi, dA.data_ptr(), K, dW.data_ptr(), K, db.data_ptr(), C.data_ptr(),
                 N, C.data_ptr() if epi == 2 else None, N, M, N, K, stream())
        outs.append(C)
    torch.cuda.synchronize()
    err = rel_err(outs[0], ref)
    assert err < (2e-3 if out_dtype == torch.float16 else 1e-4), err
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("N,K,epi", [(1536, 512, 0), (512, 512, 2), (2048, 512, 1), (512, 2048, 2)])
def test_gemm_big_bench_shapes(gpu, N, K, epi):
    """The bench's encoder projections at M = 64 x 1500 = 96 000 rows (QKV, attention output
    + residual, fc1 + GELU, fc2 + residual): bit-identical to the 128 x 128-tile kernel,
    and a sampled row block against fp64."""
    M = 96000
    g = torch.Generator(device=gpu).manual_seed(N + K)
    A = (torch.rand(M, K, device=gpu, generator=g) * 2 - 1).half()
    W = ((torch.rand(N, K, device=gpu, generator=g) * 2 - 1) / math.sqrt(K)).half()
    b = torch.randn(N, device=gpu, generator=g)
    R0 = torch.randn(M, N, device=gpu, generator=g)
    outs = []
    for fn in ("janus_gemm_f16", "janus_gemm_nt128_f16"):
        C = R0.clone() if epi == 2 else torch.empty(M, N, dtype=torch.float16, device=gpu)
        nat.call(fn, epi, A.data_ptr(), K, W.data_ptr(), K, b.data_ptr(), C.data_ptr(), N,
                 C.data_ptr() if epi == 2 else None, N, M, N, K, stream())
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    rows = torch.arange(95000, 96000, device=gpu)
    ref = A[rows].double() @ W.double().T + b.double()
    if epi == 1:
        ref = F.gelu(ref)
    if epi == 2:
        ref = ref + R0[rows].double()
    assert rel_err(outs[0][rows], ref) < (2e-3 if epi in (0, 1) else 1e-4)


@pytest.mark.parametrize("M,N,K", [(3000, 1536, 512), (3000, 512, 512), (3000, 2048, 512),
                                   (3000, 512, 2048), (1500, 384, 1536)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemm_lt(gpu, M, N, K, epi):
    """The encoder projections on hipBLASLt (janus_gemm_lt_f16): same contract as the
    hand-written GEMM, fp64 reference, in-place residual, exact-erf GELU pass."""
    g = torch.Generator().manual_seed(M + N * 3 + K + epi)
    A = (torch.randn(M, K, generator=g)).half()
    W = (torch.randn(N, K, generator=g) / math.sqrt(K)).half()
    bias = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    ref = A.double() @ W.double().T + bias.double()
    if epi == 1:
        ref = F.gelu(ref)
    if epi == 2:
        ref = ref + R.double()
    dA, dW, db = A.to(gpu), W.to(gpu), bias.to(gpu)
    out_dtype = torch.float16 if epi in (0, 1) else torch.float32
    C = R.to(gpu).clone() if epi == 2 else torch.empty(M, N, dtype=out_dtype, device=gpu)
    nat.call("janus_gemm_lt_f16", epi, dA.data_ptr(), K, dW.data_ptr(), K, db.data_ptr(), C.data_ptr(),
             N, C.data_ptr() if epi == 2 else None, N, M, N, K, stream())
    torch.cuda.synchronize()
    err = rel_err(C, ref)
    # fp16 output: one rounding (two for GELU: the library's fp16 store, then the pass)
    assert err < (2e-3 if out_dtype == torch.float16 else 1e-4), err


def test_layernorm(gpu):
    g = torch.Generator().manual_seed(1)
    for d in (384, 512, 768):
        x = torch.randn(333, d, generator=g) * 3 + 1
        gam, bet = torch.randn(d, generator=g), torch.randn(d, generator=g)
        ref = F.layer_norm(x.double(), (d,), gam.double(), bet.double(), 1e-5)
        out = torch.empty(333, d, dtype=torch.float16, device=gpu)
        dx, dg, db = x.to(gpu), gam.to(gpu), bet.to(gpu)  # keep device copies alive
        nat.call("janus_layernorm_f16", dx.data_ptr(), dg.data_ptr(), db.data_ptr(),
                 out.data_ptr(), 333, d, 1e-5, stream())
        torch.cuda.synchronize()
        assert rel_err(out, ref) < 1e-3


@pytest.mark.parametrize("B,T,H", [(2, 100, 2), (1, 1500, 6), (3, 65, 8)])
def test_attention(gpu, B, T, H):
    g = torch.Generator().manual_seed(T + H)
    d = H * 64
    qkv = (torch.randn(B, T, 3 * d, generator=g) * 1.5).half()
    q, k, v = qkv.double().split(d, dim=-1)
    q = q.view(B, T, H, 64).transpose(1, 2)
    k = k.view(B, T, H, 64).transpose(1, 2)
    v = v.view(B, T, H, 64).transpose(1, 2)
    ref = ((q @ k.transpose(-1, -2)) / 8.0).softmax(-1) @ v
    ref = ref.transpose(1, 2).reshape(B, T, d)
    out = torch.empty(B, T, d, dtype=torch.float16, device=gpu)
    dqkv = qkv.to(gpu)
    nat.call("janus_attention_f16", dqkv.data_ptr(), out.data_ptr(), B, T, H, 0.125, stream())
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 3e-3


def act(x, a):
    return {0: lambda t: t, 1: F.silu, 2: F.gelu, 3: torch.tanh}[a](x)


CONV_CASES = [
    # Cin, Cout, taps, stride, pad, dil, transposed, pre, post, res, scale, acc, T_in
    (80, 384, 3, 1, 1, 1, 0, 0, 2, False, 1.0, 0, 300),      # whisper conv1
    (384, 384, 3, 2, 1, 1, 0, 0, 2, True, 1.0, 0, 300),      # whisper conv2 (+pos)
    (512, 512, 13, 1, 6, 1, 0, 0, 0, False, 1.0, 0, 70),     # firefly conv_pre
    (256, 256, 11, 1, 25, 5, 0, 1, 1, False, 1.0, 0, 300),   # resblock c1 (pre/post SiLU)
    (128, 128, 7, 1, 9, 3, 0, 0, 0, True, 1.0, 0, 500),      # resblock c2 (+residual)
    (64, 64, 3, 1, 1, 1, 0, 1, 1, False, 1.0, 0, 700),
    (32, 32, 11, 1, 25, 5, 0, 0, 0, True, 1 / 3, 1, 900),    # parallel-block mean accumulate
    (16, 16, 7, 1, 9, 3, 0, 1, 1, False, 1.0, 0, 1000),
    (512, 256, 0, 8, 4, 1, 1, 1, 0, False, 1.0, 0, 40),      # ConvTranspose u=8 k=16
    (256, 128, 0, 8, 4, 1, 1, 1, 0, False, 1.0, 0, 50),
    (32, 16, 0, 2, 1, 1, 1, 1, 0, False, 1.0, 0, 333),       # ConvTranspose u=2 k=4
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv1d(gpu, case):
    Cin, Cout, taps, stride, pad, dil, tr, pre, post, use_res, scale, acc, T_in = case
    B = 2
    g = torch.Generator().manual_seed(Cin + Cout + taps + stride)
    x = torch.randn(B, T_in, Cin, generator=g).half()
    if tr:
        k = 2 * stride
        w = torch.randn(Cin, Cout, k, generator=g) / math.sqrt(Cin * 2)
        T_out = (T_in - 1) * stride - 2 * pad + k
    else:
        w = torch.randn(Cout, Cin, taps, generator=g) / math.sqrt(Cin * taps)
        T_out = (T_in + 2 * pad - dil * (taps - 1) - 1) // stride + 1
    bias = torch.randn(Cout, generator=g) * 0.1
    xin = act(x.double(), pre).half().double()  # kernel rounds pre-activated input to fp16
    xin = xin.transpose(1, 2)
    wq = w.half().double()
    if tr:
        ref = F.conv_transpose1d(xin, wq, bias.double(), stride=stride, padding=pad)
    else:
        ref = F.conv1d(xin, wq, bias.double(), stride=stride, padding=pad, dilation=dil)
    ref = act(ref, post).transpose(1, 2)
    res = torch.randn(B, T_out, Cout, generator=g).half() if use_res else None
    if res is not None:
        ref = ref + res.double()
    prev = torch.randn(B, T_out, Cout, generator=g).half()
    ref = ref * scale + (prev.double() if acc else 0)
    n_packed = nat.lib().janus_conv1d_packed_size(Cin, Cout, taps, tr, stride)
    packed = torch.empty(n_packed, dtype=torch.float16, device=gpu)
    dw = w.float().contiguous().to(gpu)
    nat.call("janus_conv1d_pack", dw.data_ptr(), packed.data_ptr(), Cin, Cout, taps, tr, stride, stream())
    out = prev.to(gpu).clone()
    dres = res.to(gpu) if res is not None else None
    dx, dbias = x.to(gpu), bias.to(gpu)
    nat.call("janus_conv1d_f16", dx.data_ptr(), B, T_in, Cin, packed.data_ptr(),
             dbias.data_ptr(), out.data_ptr(), T_out, Cout, taps, stride, pad, dil, tr, pre,
             post, dres.data_ptr() if dres is not None else None, T_out * Cout, scale, acc, stream())
    torch.cuda.synchronize()
    assert out.shape == ref.shape
    err = rel_err(out, ref)
    assert err < 2e-3, err


@pytest.mark.parametrize("C,k,d,acc,T", [(16, 3, 1, 0, 1500), (16, 11, 5, 1, 1500), (32, 7, 3, 0, 1500),
                                         (32, 11, 5, 1, 1500), (16, 7, 1, 1, 1500), (32, 3, 3, 0, 1500),
                                         (64, 3, 1, 0, 1500), (64, 11, 5, 1, 1500), (64, 7, 3, 1, 37),
                                         (128, 7, 3, 1, 1500), (128, 11, 5, 0, 1500), (128, 3, 1, 1, 129),
                                         (256, 3, 1, 1, 700), (256, 11, 5, 0, 700), (256, 7, 3, 1, 20)])
def test_resunit(gpu, C, k, d, acc, T):
    B = 2
    g = torch.Generator().manual_seed(C * 100 + k * 10 + d)
    x = torch.randn(B, T, C, generator=g).half()
    w1 = torch.randn(C, C, k, generator=g) / math.sqrt(C * k)
    w2 = torch.randn(C, C, k, generator=g) / math.sqrt(C * k)
    b1 = torch.randn(C, generator=g) * 0.1
    b2 = torch.randn(C, generator=g) * 0.1
    prev = torch.randn(B, T, C, generator=g).half()
    scale = 1 / 3 if acc else 1.0
    xd = x.double().transpose(1, 2)
    h = F.conv1d(F.silu(xd).half().double(), w1.half().double(), b1.double(), padding=d * (k - 1) // 2,
                 dilation=d)
    h = F.silu(h).half().double()
    y = F.conv1d(h, w2.half().double(), b2.double(), padding=(k - 1) // 2) + xd
    ref = y.transpose(1, 2) * scale + (prev.double() if acc else 0)
    n = nat.lib().janus_resunit_packed_size(C, k)
    p1 = torch.empty(n, dtype=torch.float16, device=gpu)
    p2 = torch.empty(n, dtype=torch.float16, device=gpu)
    dw1, dw2 = w1.to(gpu), w2.to(gpu)
    nat.call("janus_resunit_pack", dw1.data_ptr(), p1.data_ptr(), C, k, stream())
    nat.call("janus_resunit_pack", dw2.data_ptr(), p2.data_ptr(), C, k, stream())
    dx, db1, db2 = x.to(gpu), b1.to(gpu), b2.to(gpu)
    out = prev.to(gpu).clone()
    nat.call("janus_resunit_f16", dx.data_ptr(), out.data_ptr(), p1.data_ptr(), db1.data_ptr(),
             p2.data_ptr(), db2.data_ptr(), B, T, C, k, d, scale, acc, stream())
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 2e-3


@pytest.mark.parametrize("B,Te,D,nsplit", [(2, 1500, 512, 8), (3, 100, 384, 3), (1, 77, 768, 1),
                                            (4, 1500, 512, 63), (5, 1500, 512, 1), (3, 130, 384, 1)])
def test_cross_attention_absorbed(gpu, B, Te, D, nsplit):
    """softmax_2(qk_h . enc^T) . enc per head vs a float64 torch reference (nsplit 1 at D <=
    512: the kernel writes c itself, no merge launch)."""
    H = D // 64
    g = torch.Generator().manual_seed(B * 1000 + Te + D)
    enc = torch.randn(B, Te, D, generator=g).half()
    qk = (torch.randn(B, H, D, generator=g) * 0.15).half()
    s = torch.einsum("bhd,btd->bht", qk.double(), enc.double())
    p = torch.softmax(s * math.log(2.0), dim=-1)
    ref = torch.einsum("bht,btd->bhd", p, enc.double()).reshape(B, H * D)
    dq, de = qk.to(gpu), enc.to(gpu)
    pc = torch.empty(B * nsplit * H * D, dtype=torch.float32, device=gpu)
    pml = torch.empty(B * nsplit * H * 2, dtype=torch.float32, device=gpu)
    out = torch.empty(B, H * D, dtype=torch.float16, device=gpu)
    nat.call("janus_cross_attention_f16", dq.data_ptr(), de.data_ptr(), B, Te, D, H, nsplit,
             pc.data_ptr(), pml.data_ptr(), out.data_ptr(), stream())
    torch.cuda.synchronize()
    err = rel_err(out, ref)
    assert err < 3e-3, err


@pytest.mark.parametrize("B,T,H,split", [(3, 1, 8, 0), (2, 37, 6, 0), (64, 448, 8, 0), (2, 512, 8, 0),
                                         (2, 700, 8, 1), (3, 1000, 8, 1)])
def test_decode_attention(gpu, B, T, H, split):
    """One query per (b, h) against a KV cache with row stride > d (the decoder's cache
    layout [B][n_ctx][d]); per-head kernel (T <= 512) and the key-split + combine path."""
    d, n_ctx = H * 64, max(T, 448) + 5
    g = torch.Generator().manual_seed(B * 100 + T + H)
    q = (torch.randn(B, 3 * d, generator=g)).half()          # q is the first d of a qkv row
    k = (torch.randn(B, n_ctx, d, generator=g)).half()
    v = (torch.randn(B, n_ctx, d, generator=g)).half()
    qh = q[:, :d].double().view(B, H, 1, 64)
    kh = k[:, :T].double().view(B, T, H, 64).transpose(1, 2)
    vh = v[:, :T].double().view(B, T, H, 64).transpose(1, 2)
    ref = (((qh @ kh.transpose(-1, -2)) * 0.125).softmax(-1) @ vh).reshape(B, d)
    dq, dk, dv = q.to(gpu), k.to(gpu), v.to(gpu)
    out = torch.empty(B, 2 * d, dtype=torch.float16, device=gpu)
    ns = (T + 63) // 64
    po = torch.empty(B * ns * d, dtype=torch.float32, device=gpu) if split or T > 512 else None
    pm = torch.empty(B * ns * H * 2, dtype=torch.float32, device=gpu) if split or T > 512 else None
    nat.call("janus_decode_attention_f16", dq.data_ptr(), 3 * d, dk.data_ptr(), dv.data_ptr(),
             n_ctx * d, d, T, out.data_ptr(), 2 * d, B, H, 0.125,
             po.data_ptr() if po is not None else None, pm.data_ptr() if pm is not None else None,
             stream())
    torch.cuda.synchronize()
    err = rel_err(out[:, :d], ref)
    assert err < 2e-3, err


@pytest.mark.parametrize("M,N,epi", [(64, 1536, 0), (64, 4096, 0), (37, 2048, 1), (5, 512, 0)])
def test_gemm_layernorm_prologue(gpu, M, N, epi):
    """epilogue(LayerNorm(x) W^T + b) with the LayerNorm in the GEMM prologue vs float64."""
    K = 512
    g = torch.Generator().manual_seed(M + N + epi)
    x = torch.randn(M, K, generator=g) * 2.0 + 0.5
    gam = torch.randn(K, generator=g) * 0.2 + 1.0
    bet = torch.randn(K, generator=g) * 0.1
    W = (torch.randn(N, K, generator=g) / math.sqrt(K)).half()
    bias = torch.randn(N, generator=g) * 0.1
    xn = F.layer_norm(x.double(), (K,), gam.double(), bet.double(), 1e-5)
    ref = xn.half().double() @ W.double().T + bias.double()
    if epi == 1:
        ref = F.gelu(ref)
    out = torch.empty(M, N, dtype=torch.float16, device=gpu)
    dx, dg, db, dW, dbias = x.to(gpu), gam.to(gpu), bet.to(gpu), W.to(gpu), bias.to(gpu)
    nat.call("janus_gemm_ln_f16", epi, dx.data_ptr(), K, dg.data_ptr(), db.data_ptr(), 1e-5,
             dW.data_ptr(), K, dbias.data_ptr(), out.data_ptr(), N, M, N, K, stream())
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 2e-3


@pytest.mark.parametrize("M,d", [(64, 512), (37, 512), (5, 384), (64, 384)])
def test_resid_ln_matches_two_launches(gpu, M, d):
    """janus_resid_ln_f16 (the decoder's attention output projection + the following
    LayerNorm in one launch) is bit-identical to the residual skinny GEMM followed by the
    LayerNorm launch it replaces, and within fp32 rounding of a float64 reference."""
    g = torch.Generator().manual_seed(M + d)
    A = torch.randn(M, d, generator=g).half()
    W = (torch.randn(d, d, generator=g) / math.sqrt(d)).half()
    bias = torch.randn(d, generator=g) * 0.1
    x0 = torch.randn(M, d, generator=g) * 2.0 + 0.3
    gam = torch.randn(d, generator=g) * 0.2 + 1.0
    bet = torch.randn(d, generator=g) * 0.1
    dA, dW, db, dg, dbt = A.to(gpu), W.to(gpu), bias.to(gpu), gam.to(gpu), bet.to(gpu)
    # two launches
    x1 = x0.to(gpu)
    out1 = torch.empty(M, d, dtype=torch.float16, device=gpu)
    nat.call("janus_gemm_f16", 2, dA.data_ptr(), d, dW.data_ptr(), d, db.data_ptr(), x1.data_ptr(), d,
             x1.data_ptr(), d, M, d, d, stream())
    nat.call("janus_layernorm_f16", x1.data_ptr(), dg.data_ptr(), dbt.data_ptr(), out1.data_ptr(), M, d,
             1e-5, stream())
    # one launch
    x2 = x0.to(gpu)
    out2 = torch.empty(M, d, dtype=torch.float16, device=gpu)
    nat.call("janus_resid_ln_f16", dA.data_ptr(), d, dW.data_ptr(), d, db.data_ptr(), x2.data_ptr(),
             dg.data_ptr(), dbt.data_ptr(), 1e-5, out2.data_ptr(), M, d, d, stream())
    torch.cuda.synchronize()
    assert torch.equal(x1, x2)
    assert torch.equal(out1, out2)
    ref_x = x0.double() + A.double() @ W.double().T + bias.double()
    assert rel_err(x2, ref_x) < 1e-6
    ref = F.layer_norm(ref_x, (d,), gam.double(), bet.double(), 1e-5)
    assert rel_err(out2, ref) < 1e-3


@pytest.mark.parametrize("M,N", [(64, 4096), (64, 1536), (37, 2304)])
def test_gemm_layernorm_prologue_bit_identical(gpu, M, N):
    """A LayerNorm in the GEMM prologue (janus_gemm_ln_f16, the decoder's pre-LN
    projections) rounds exactly as the LayerNorm launch followed by the plain GEMM."""
    K = 512
    g = torch.Generator().manual_seed(M * 3 + N)
    x = torch.randn(M, K, generator=g) * 2.0 + 0.5
    gam = torch.randn(K, generator=g) * 0.2 + 1.0
    bet = torch.randn(K, generator=g) * 0.1
    W = (torch.randn(N, K, generator=g) / math.sqrt(K)).half()
    bias = torch.randn(N, generator=g) * 0.1
    dx, dg, db, dW, dbias = x.to(gpu), gam.to(gpu), bet.to(gpu), W.to(gpu), bias.to(gpu)
    out1 = torch.empty(M, N, dtype=torch.float16, device=gpu)
    nat.call("janus_gemm_ln_f16", 0, dx.data_ptr(), K, dg.data_ptr(), db.data_ptr(), 1e-5,
             dW.data_ptr(), K, dbias.data_ptr(), out1.data_ptr(), N, M, N, K, stream())
    a = torch.empty(M, K, dtype=torch.float16, device=gpu)
    nat.call("janus_layernorm_f16", dx.data_ptr(), dg.data_ptr(), db.data_ptr(), a.data_ptr(), M, K,
             1e-5, stream())
    out2 = torch.empty(M, N, dtype=torch.float16, device=gpu)
    nat.call("janus_gemm_f16", 0, a.data_ptr(), K, dW.data_ptr(), K, dbias.data_ptr(), out2.data_ptr(), N,
             None, N, M, N, K, stream())
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)


def test_wave_xor_shuffles(gpu):
    """mfma.h xshfl<O> (DPP quad_perm / row_ror / row_shl+shr, v_permlane16/32_swap): every
    lane receives exactly lane ^ O's value, so the butterfly reductions built on it
    (softmax, LayerNorm) keep __shfl_xor's association bit for bit."""
    n = 4
    x = torch.randn(n, 64, generator=torch.Generator().manual_seed(7))
    dx = x.to(gpu)
    out = torch.empty(n, 6, 64, device=gpu)
    nat.call("janus_wave_xor_f32", dx.data_ptr(), out.data_ptr(), n, stream())
    torch.cuda.synchronize()
    lanes = torch.arange(64)
    for k in range(6):
        assert torch.equal(out[:, k].cpu(), x[:, lanes ^ (1 << k)]), k
