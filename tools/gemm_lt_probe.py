"""Encoder projection shapes (64 x 1500 rows, base.en) on gemm_nt_kernel vs hipBLASLt
(janus_gemm_f16 vs janus_gemm_lt_f16), microseconds per call, one JSON line each."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from janus_amd import _native as nat
    dev = torch.device("cuda", 0)
    M = 96000
    for name, N, K, epi in [("qkv", 1536, 512, 0), ("o_resid", 512, 512, 2), ("fc1_gelu", 2048, 512, 1),
                            ("fc2_resid", 512, 2048, 2)]:
        A = torch.randn(M, K, device=dev).half()
        W = (torch.randn(N, K, device=dev) / math.sqrt(K)).half()
        b = torch.randn(N, device=dev)
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if epi == 2 else torch.float16)
        s = torch.cuda.current_stream().cuda_stream
        res = {"gemm": name, "M": M, "N": N, "K": K}
        outs = {}
        for fn in ("janus_gemm_f16", "janus_gemm_lt_f16"):
            C.zero_()
            def run():
                nat.call(fn, epi, A.data_ptr(), K, W.data_ptr(), K, b.data_ptr(), C.data_ptr(), N,
                         C.data_ptr() if epi == 2 else None, N, M, N, K, s)
            run()
            torch.cuda.synchronize()
            outs[fn] = C.float().clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 100
            res[fn.replace("janus_", "") + "_us"] = round(us, 1)
            res[fn.replace("janus_", "") + "_tflops"] = round(2.0 * M * N * K / us / 1e6, 1)
        a, c = outs["janus_gemm_f16"], outs["janus_gemm_lt_f16"]
        res["rel_diff"] = float((a - c).norm() / (a.norm() + 1e-30))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
