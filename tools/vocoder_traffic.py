"""HBM traffic of the vocoder's conv launches (the bench's roofline kernel).

Run under two rocprofv3 PMC passes (FETCH_SIZE, then WRITE_SIZE):
  rocprofv3 --kernel-trace --pmc FETCH_SIZE -d out/f -o run --output-format csv -- python3 tools/vocoder_traffic.py
then ``python3 tools/vocoder_traffic.py --reduce out/f out/w profiles/traffic_r01.json`` sums the
counters over the conv dispatches of the profiled forward (one 64 x 30 s batch, the bench
workload) and writes bytes per launch, with the gfx950 correction (FETCH_SIZE reports half
of the bytes of 16-B-per-lane streaming reads: MI355X_MICROARCH.md 'HBM').
"""
import csv
import glob
import json
import os
import sys


def run():
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from janus_amd.vocoder import VocoderEngine, emotion_id
    eng = VocoderEngine()
    B, F = 64, 2584
    prompts = [b"(relaxed) traffic sample %d" % i for i in range(B)]
    lat = eng.frontend(prompts, [emotion_id("relaxed")] * B, F)
    eng.set_timing(True)
    eng.forward(lat)
    torch.cuda.synchronize()
    flops, ms, launches = eng.conv_stats(reset=True)
    print(json.dumps({"conv_flops": flops, "conv_ms": ms, "conv_launches": launches}))


def family(k):
    """Kernel name -> vocoder family: the channel width of a fused unit, or 'conv'."""
    import re
    m = re.search(r"resunit(?:_wide)?(?:_lds)?_kernel<(\d+)", k)
    if m:
        return int(m.group(1))
    return "conv" if "conv_kernel" in k else None


def counters(d, by_family=False):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    tot, n = 0.0, set()
    fam = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "conv_kernel" in k or ("resunit" in k and "pack" not in k):
            tot += float(r["Counter_Value"])
            n.add(r["Dispatch_Id"])
            g = fam.setdefault(str(family(k)), [0.0, set()])
            g[0] += float(r["Counter_Value"])
            g[1].add(r["Dispatch_Id"])
    if by_family:
        return {k: (v[0], len(v[1])) for k, v in fam.items()}
    return tot, len(n)


def algorithmic_bytes(B=64, F=2584, latent=512, ch=512, ups=(8, 8, 2, 2, 2), n_k=3, n_d=3,
                      by_family=False):
    """Bytes each conv / fused-unit launch of one forward must move at least (fp16 tensors
    read once, written once), following vocoder.cpp forward: (launches, total bytes), or
    per family {C or 'conv': (launches, bytes)}."""
    fam = {}

    def add(key, b):
        f = fam.setdefault(str(key), [0, 0])
        f[0] += 1
        f[1] += b
    T = F
    add("conv", 2 * B * (F * latent + F * ch))            # conv_pre
    c = ch
    for u in ups:
        add("conv", 2 * B * (T * c + T * u * (c // 2)))    # ConvTranspose
        T *= u
        c //= 2
        for kj in range(n_k):
            for m in range(n_d):
                last = m + 1 == n_d
                acc = last and kj > 0
                add(c, 2 * B * T * c * (2 + (1 if acc else 0)))  # fused unit: x in, out (+ acc read)
    if by_family:
        return {k: tuple(v) for k, v in fam.items()}
    return sum(v[0] for v in fam.values()), sum(v[1] for v in fam.values())


def reduce(fdir, wdir, out):
    fetch_kb, nf = counters(fdir)
    write_kb, nw = counters(wdir)
    assert nf == nw and nf > 0, (nf, nw)
    fetch = 2.0 * fetch_kb * 1024  # gfx950: FETCH_SIZE = half the streamed bytes (KB units)
    write = write_kb * 1024
    res = {"kernel": "conv_kernel + resunit_kernel + resunit_wide[_lds]_kernel (vocoder convs, all shapes of one 64 x 30 s "
                     "forward: the launch set the bench's roofline averages over)",
           "launches": nf, "fetch_bytes": fetch, "write_bytes": write,
           "bytes_per_launch": (fetch + write) / nf,
           "algorithmic_bytes_per_launch": algorithmic_bytes()[1] / algorithmic_bytes()[0],
           "algorithmic_launches": algorithmic_bytes()[0],
           "correction": "FETCH_SIZE x2 (gfx950 wide-read under-count), KB -> bytes x1024",
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes"}
    ff, fw, alg = counters(fdir, True), counters(wdir, True), algorithmic_bytes(by_family=True)
    res["by_family"] = {
        k: {"launches": ff[k][1], "fetch_bytes": 2.0 * ff[k][0] * 1024, "write_bytes": fw[k][0] * 1024,
            "algorithmic_bytes": alg[k][1],
            "traffic_over_algorithmic": (2.0 * ff[k][0] + fw[k][0]) * 1024 / alg[k][1]}
        for k in sorted(ff, key=str) if k in alg}
    res["traffic_over_algorithmic"] = res["bytes_per_launch"] / res["algorithmic_bytes_per_launch"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--reduce":
        reduce(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        run()
