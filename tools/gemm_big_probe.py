"""Encoder projection shapes (64 x 1500 rows, base.en): the 256x256-tile kernel
(janus_gemm_f16 -> gemm_big), the 128x128-tile kernel (janus_gemm_nt128_f16) and hipBLASLt
(janus_gemm_lt_f16): microseconds per call, TF/s, and bit-identity big vs nt128."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from janus_amd import _native as nat
    dev = torch.device("cuda", 0)
    M = int(os.environ.get("GEMM_M", "96000"))
    fns = os.environ.get("GEMM_FNS", "janus_gemm_f16,janus_gemm_nt128_f16,janus_gemm_lt_f16").split(",")
    for name, N, K, epi in [("qkv", 1536, 512, 0), ("o_resid", 512, 512, 2), ("fc1_gelu", 2048, 512, 1),
                            ("fc2_resid", 512, 2048, 2)]:
        g = torch.Generator(device=dev).manual_seed(N + K)
        A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).half()
        W = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) / math.sqrt(K)).half()
        b = torch.randn(N, device=dev, generator=g)
        R0 = torch.randn(M, N, device=dev, generator=g)
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if epi == 2 else torch.float16)
        s = torch.cuda.current_stream().cuda_stream
        res = {"gemm": name, "M": M, "N": N, "K": K}
        outs = {}
        for fn in fns:
            def run():
                nat.call(fn, epi, A.data_ptr(), K, W.data_ptr(), K, b.data_ptr(), C.data_ptr(), N,
                         C.data_ptr() if epi == 2 else None, N, M, N, K, s)
            if epi == 2:
                C.copy_(R0)
            else:
                C.zero_()
            try:
                run()
            except Exception as e:  # no library plan
                res[fn] = repr(e)[:80]
                continue
            torch.cuda.synchronize()
            outs[fn] = C.float().clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000 / 20
            res[fn.replace("janus_", "") + "_us"] = round(us, 1)
            res[fn.replace("janus_", "") + "_tflops"] = round(2.0 * M * N * K / us / 1e6, 1)
        # JANUS_GEMM_BIG schedules A/B'd in one process, interleaved rounds (the variant is
        # read per launch): median and min microseconds, bit-identity with the default
        for v in [x for x in os.environ.get("GEMM_VARIANTS", "").split(",") if x]:
            os.environ["JANUS_GEMM_BIG"] = v
            if epi == 2:
                C.copy_(R0)
            else:
                C.zero_()
            run()
            torch.cuda.synchronize()
            res["eq_" + v] = bool(torch.equal(C.float(), outs.get("janus_gemm_f16", C.float())))
        rounds = {}
        for r in range(int(os.environ.get("GEMM_ROUNDS", "5")) if os.environ.get("GEMM_VARIANTS") else 0):
            for v in [x for x in os.environ["GEMM_VARIANTS"].split(",") if x]:
                os.environ["JANUS_GEMM_BIG"] = v
                def run_v():
                    nat.call("janus_gemm_f16", epi, A.data_ptr(), K, W.data_ptr(), K, b.data_ptr(),
                             C.data_ptr(), N, C.data_ptr() if epi == 2 else None, N, M, N, K, s)
                run_v()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    run_v()
                e1.record()
                torch.cuda.synchronize()
                rounds.setdefault(v, []).append(e0.elapsed_time(e1) * 100)
        os.environ.pop("JANUS_GEMM_BIG", None)
        for v, ts in rounds.items():
            ts.sort()
            res[v + "_us_median"] = round(ts[len(ts) // 2], 1)
            res[v + "_us_min"] = round(ts[0], 1)
            res[v + "_tflops_median"] = round(2.0 * M * N * K / ts[len(ts) // 2] / 1e6, 1)
        if "janus_gemm_f16" in outs and "janus_gemm_nt128_f16" in outs:
            res["big_eq_nt128"] = bool(torch.equal(outs["janus_gemm_f16"], outs["janus_gemm_nt128_f16"]))
        if "janus_gemm_f16" in outs and "janus_gemm_lt_f16" in outs:
            a, c = outs["janus_gemm_f16"], outs["janus_gemm_lt_f16"]
            res["rel_diff_vs_lt"] = float((a - c).norm() / (a.norm() + 1e-30))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
