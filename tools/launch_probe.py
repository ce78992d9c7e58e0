"""Per-launch cost of the decoder's small kernels, outside the decoder: chains of N
dependent launches captured in one HIP graph (torch.cuda.graph over the C-ABI entry
points), replayed on a CU-masked stream of `per_xcd` CUs per XCD (16 = the overlapped
step's decoder partition) or every CU (0 / 32: an all-ones mask through the same stream API). Prints one JSON line per chain:
microseconds per launch. Chains: LayerNorm alone (64 x 512 rows), the residual projection
alone (64 x 512 x 512), and the decoder's pair residual projection -> LayerNorm.

python tools/launch_probe.py [--per-xcd 16] [--n 200]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-xcd", type=int, default=16)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--plain", type=int, default=0, help="1: an ordinary torch stream, no CU mask")
    ap.add_argument("--priority", type=int, default=0, help="torch stream priority (plain only)")
    a = ap.parse_args()
    import torch
    from janus_amd import _native as nat
    lib = nat.lib()
    dev = torch.device("cuda", 0)
    M, D = 64, 512
    x = torch.randn(M, D, device=dev)
    g = torch.ones(D, device=dev)
    b = torch.zeros(D, device=dev)
    a16 = torch.zeros(M, D, dtype=torch.float16, device=dev)
    W = (torch.randn(D, D, device=dev) * 0.02).half()
    bias = torch.zeros(D, device=dev)
    EPI_RESID_F32 = 2
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    if a.plain:
        stream = torch.cuda.Stream(dev, priority=a.priority)
    elif 0 < a.per_xcd < n // 8:
        dmask, _ = nat.split_cu_masks(n, a.per_xcd)
    else:  # every CU, through the same CU-masked stream API
        dmask = [0xFFFFFFFF] * (n // 32)
    if not a.plain:
        ms = nat.MaskedStream(dmask, dev)
        stream = ms.stream
    sp = ctypes.c_void_p(stream.cuda_stream)

    def ln():
        nat.call("janus_layernorm_f16", ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(g.data_ptr()),
                 ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(a16.data_ptr()), M, D,
                 ctypes.c_float(1e-5), sp)

    def resid():
        nat.call("janus_gemm_f16", EPI_RESID_F32, ctypes.c_void_p(a16.data_ptr()), D,
                 ctypes.c_void_p(W.data_ptr()), D, ctypes.c_void_p(bias.data_ptr()),
                 ctypes.c_void_p(x.data_ptr()), D, ctypes.c_void_p(x.data_ptr()), D, M, D, D, sp)

    W0 = torch.zeros(D, D, dtype=torch.float16, device=dev)
    ones = torch.ones(D, device=dev)
    xc = torch.zeros(M, D, device=dev)

    def count():  # xc += 0 . a + 1: lost updates if two launches of the chain overlap
        nat.call("janus_gemm_f16", EPI_RESID_F32, ctypes.c_void_p(a16.data_ptr()), D,
                 ctypes.c_void_p(W0.data_ptr()), D, ctypes.c_void_p(ones.data_ptr()),
                 ctypes.c_void_p(xc.data_ptr()), D, ctypes.c_void_p(xc.data_ptr()), D, M, D, D, sp)

    chains = {"layernorm": [ln], "resid_gemm": [resid], "resid_gemm+layernorm": [resid, ln],
              "ordered_count": [count]}
    for name, ops in chains.items():
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream):
            for op in ops:  # warm (attributes, first-launch setup) outside the capture
                op()
            torch.cuda.synchronize()
            with torch.cuda.graph(gr, stream=stream):
                for _ in range(a.n):
                    for op in ops:
                        op()
        torch.cuda.synchronize()
        if ops[-1] is count:  # launches of the chain run in order, none overlapping
            xc.zero_()
            torch.cuda.synchronize()
            with torch.cuda.stream(stream):
                gr.replay()
            torch.cuda.synchronize()
            got = float(xc.min().item()), float(xc.max().item())
            assert got == (float(a.n), float(a.n)), f"chain not serialised: {got} vs {a.n}"
        if ops[-1] is ln:  # the replay really runs the captured launches
            a16.zero_()
            torch.cuda.synchronize()
            with torch.cuda.stream(stream):
                gr.replay()
            torch.cuda.synchronize()
            assert a16.abs().sum().item() > 0, "replay did not run the captured launches"
        best = None
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):  # replay() launches on the current stream
                e0.record(stream)
                gr.replay()
                e1.record(stream)
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) * 1e3 / (a.n * len(ops))
            best = t if best is None else min(best, t)
        print(json.dumps({"chain": name, "per_xcd": a.per_xcd, "plain": a.plain, "priority": a.priority,
                          "packet_capture": os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE"), "launches": a.n * len(ops),
                          "us_per_launch": round(best, 2)}), flush=True)


if __name__ == "__main__":
    main()
