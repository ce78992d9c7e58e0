"""Per-kernel roofline of the greedy decoder from a rocprofv3 kernel-stats CSV (the bench's
overlapped step: base.en, 64 utterances, 447 positions per decode; the decoder runs inside
HIP graphs, so per-launch HIP events are not available and rocprof's average duration is
the clock).

python tools/decoder_roofline.py profiles/r02_v6_kernel_stats.csv [--json out.json]

Algorithmic bytes per launch (fp16 = 2 B), B = 64, d = 512, H = 8, Te = 1500, V = 51864:
  xattn_kernel          encoder output read once: B*Te*d*2
  decode_head_kernel<NR> K and V cache rows of the keys that exist: B*H*Tkv*64*2*2, with
                        Tkv averaged over the positions whose key count falls in round NR
  logits_partial        tied embedding: V*d*2 (+ A, negligible)
  skinny projections    weights N*K*2 (+ A and outputs, small)
Peak: 8 TB/s HBM (MI355X_MICROARCH.md); the decoder owns half the CUs beside the vocoder,
so the fraction is also given against that half's share (4 TB/s).
"""
import argparse
import csv
import json
import re

B, D, H, TE, V, POS = 64, 512, 8, 1500, 51864, 447
PEAK = 8000.0  # GB/s


def head_bytes(nr):
    # positions p = 0..446 attend over Tkv = p + 1 keys; round NR holds Tkv in (64(NR-1), 64 NR]
    ts = [t for t in range(1, POS + 1) if (t + 63) // 64 == nr]
    if not ts:
        return None
    return B * H * (sum(ts) / len(ts)) * 64 * 2 * 2


def classify(name):
    if "xattn_kernel" in name:
        return "cross-attention (xattn_kernel)", B * TE * D * 2
    m = re.search(r"decode_head_kernelILi(\d+)E", name)
    if m:
        nr = int(m.group(1))
        return f"self-attention (decode_head_kernel<{nr}>)", head_bytes(nr)
    if "logits_partial_kernel" in name:
        return "vocabulary projection (logits_partial)", V * D * 2
    if "gemm_skinny2_kernel" in name:
        return "absorbed query projection (gemm_skinny2, N 4096)", 4096 * D * 2
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--json")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        fam, by = classify(r["Name"])
        if fam is None or by is None:
            continue
        avg_us = float(r["AverageNs"]) / 1000.0
        gbs = by / (avg_us * 1e-6) / 1e9
        rows.append(dict(kernel=fam, calls=int(r["Calls"]), avg_us=round(avg_us, 2),
                         mb_per_launch=round(by / 1e6, 2), gbs=round(gbs, 1),
                         frac_of_peak=round(gbs / PEAK, 3), frac_of_half=round(gbs / (PEAK / 2), 3)))
    for x in rows:
        print(f"{x['kernel']:55s} {x['calls']:6d} calls {x['avg_us']:8.2f} us {x['mb_per_launch']:8.2f} MB "
              f"{x['gbs']:8.1f} GB/s  {x['frac_of_peak']:.3f} of 8 TB/s, {x['frac_of_half']:.3f} of the half share")
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
