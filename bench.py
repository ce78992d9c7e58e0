"""Janus hot-path benchmark: end-to-end encode + decode xRT on MI355X.

Workload (BASELINE.json metric "xRT (audio-s/wall-s) per GPU, 30s clips batch=64"):
per GPU, 64 seeded synthetic 30 s utterances at 48 kHz (janus_amd/workload.py) already
resident in HBM. One step = the whole batch through
  encode: log-mel([::3]) -> Whisper base.en encoder -> greedy decoder (<= 448 tokens,
          timestamp rules) -> detokenize -> YIN + RMS prosody -> MessagePack packets
  decode: unpack -> "(emotion) text" prompt -> front end -> Firefly-GAN vocoder
          (30 s = 2584 latent frames -> 1 323 008 samples @ 44.1 kHz, f32 + int16)
Default (--overlap 16): the steady-state serving pipeline — each step encodes batch i
and renders the packets of batch i-1, so every timed step carries one full encode and
one full decode of 64 utterances (a warm-up step primes it). After the encoder, the
greedy decoder runs on 16 CUs of each XCD and the vocoder + YIN on the other 16
(CU-masked streams). --overlap 0 runs encode and decode of one batch back to back.
Weights are seeded synthetic tensors of the real shapes (no checkpoints offline).
Multi-GPU: one process per GPU, utterances sharded with no data-path collective; packet
bytes are all-gathered once after the timed steps (RCCL over xGMI).

Prints ONE JSON line on rank 0 (contract in the task statement), with a
``roofline`` object for the dominant kernel (the vocoder's implicit-GEMM MFMA conv,
timed live with HIP events on its stream) and a ``cpu_baseline`` object (the oracle's
CPU restatement on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MFMA_F16_PEAK_TFLOPS = 2500.0   # dense fp16 MFMA, MI355X_MICROARCH.md
AUDIO_SECONDS = 30.0
FRAMES_30S = 2584               # 30 s * 44100 / 512 (rounded up)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=64, help="utterances per GPU")
    ap.add_argument("--seconds", type=float, default=AUDIO_SECONDS)
    ap.add_argument("--model", default="base.en")
    ap.add_argument("--max-length", type=int, default=448)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--overlap", type=int, default=int(os.environ.get("JANUS_OVERLAP", "16")),
                    help="CUs per XCD (of 32) for the greedy decoder in the overlapped serving step "
                         "(vocoder of batch i-1 on the rest; multiples of 4 keep every shader engine "
                         "even); 0 = sequential step")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r03.json"))
    ap.add_argument("--fallback", action="store_true",
                    help="run faster-whisper's temperature fallback on windows failing their gates "
                         "(generate_with_fallback: 5 temperatures x best_of 5 sampled re-decodes); "
                         "off by default: the seeded synthetic weights fail every window (DESIGN.md §0)")
    return ap.parse_args()


def cpu_baseline(model: str, tokens_per_utt: float):
    """Oracle (CPU restatement) time for ONE whole 30 s utterance of the workload, every
    stage measured, nothing scaled: log-mel of the clip, the encoder on its window, the
    sequential KV-cache greedy loop for as many tokens as the GPU emitted per utterance
    (the reference's decode loop shape), YIN over all 30 s, and the vocoder for the
    30 s (2584 latent frames). ~10-30 s of CPU work."""
    from janus_amd import vocoder as jv
    from janus_amd import whisper as jw
    from janus_amd.tokenizer import load_tokenizer
    from janus_amd.workload import synth_speech
    from oracle import prosody as op
    from oracle import vocoder as ov
    from oracle import whisper as ow
    affinity = len(os.sched_getaffinity(0))
    # every host CPU this process may use: the affinity set, capped by OMP_NUM_THREADS when
    # the machine sets it (the GPU boxes allot 16 host CPUs per GPU and export 16 there,
    # while the affinity mask shows the whole host)
    threads = min(affinity, int(os.environ.get("OMP_NUM_THREADS", affinity)))
    torch.set_num_threads(threads)
    cfg = jw.CONFIGS[model]
    W = jw.synthetic_weights(cfg, 0)
    tk = load_tokenizer()
    x = synth_speech(999, AUDIO_SECONDS)
    n_tok = max(1, int(round(tokens_per_utt)))
    t = {}
    t0 = time.perf_counter()
    mel = ow.logmel(x, 3, jw.mel_filters())
    t["mel"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    enc = ow.encoder(mel[None], W, cfg)
    t["encoder"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    dec = ow.greedy_cached(enc.half().float(), W, cfg, tk, max_length=len(tk.sot_sequence) + n_tok)
    t["decoder"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    op.yin_stream(x)
    t["prosody"] = time.perf_counter() - t0
    vc = jv.FireflyConfig()
    VW = jv.synthetic_weights(vc, 0)
    lat = ov.frontend([b"(auto) sample"], [jv.emotion_id("auto")], FRAMES_30S, VW)
    t0 = time.perf_counter()
    ov.generator(lat, VW, vc)
    t["vocoder"] = time.perf_counter() - t0
    total = sum(t.values())
    return {
        "value": AUDIO_SECONDS / total,
        "unit": "xRT (audio-s/wall-s)",
        "cores": threads,
        "kind": "port",
        "sample": ("oracle CPU restatement (numpy/torch fp32 + C YIN), one whole 30 s utterance, "
                   f"every stage measured: mel, encoder window, sequential KV-cache greedy loop "
                   f"over {len(dec[0]['tokens'])} tokens, YIN over 30 s (1 thread), vocoder 30 s "
                   f"({FRAMES_30S} frames)"),
        "stage_seconds": {k: round(v, 3) for k, v in t.items()},
        "affinity_cpus": affinity,
        "cores_note": ("threads = min(affinity, OMP_NUM_THREADS): the host CPU share this GPU's "
                       "process is given (16 per GPU on the bench boxes, whose affinity mask "
                       "lists the whole host)"),
        "cpu_model": _cpu_model(),
    }


HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md (spec; 6.3 TB/s measured copy)


def family_lines(fams, cu_share):
    out = []
    for f, v in sorted(fams.items()):
        if v["ms"] <= 0:
            continue
        tf = v["flops"] / (v["ms"] * 1e-3) / 1e12
        gbs = v["bytes"] / (v["ms"] * 1e-3) / 1e9
        mf = tf / (MFMA_F16_PEAK_TFLOPS * cu_share)
        hf = gbs / (HBM_PEAK_GBS * cu_share)
        out.append({"family": "conv" if f == 0 else f"unit C={f}", "launches": v["launches"],
                    "ms": round(v["ms"], 2), "achieved_tflops": round(tf, 1),
                    "mfma_frac_of_share": round(mf, 3), "hbm_gbs_algorithmic": round(gbs, 1),
                    "hbm_frac_of_share": round(hf, 3), "bound": "mfma" if mf >= hf else "hbm"})
    return out


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    # JANUS_DIST_FORCE=1: the RCCL path (process group, barriers, max-over-ranks all-reduce,
    # result gather) at world size 1 too — exercises it on a one-GPU box
    use_dist = world > 1 or os.environ.get("JANUS_DIST_FORCE") == "1"
    if use_dist:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from janus_amd.dist import gather_results, shard
    from janus_amd.pipeline import JanusPipeline
    from janus_amd.workload import synth_speech

    dev = torch.device("cuda", local)
    # weak scaling: B utterances per GPU; rank r owns shard(r) of the job's world*B
    # utterances (seed = 1000*config + global index, config 4)
    u0, u1 = shard(rank, world, world * args.batch)
    B = u1 - u0
    utts = [synth_speech(4000 + i, args.seconds) for i in range(u0, u1)]
    lengths = [len(u) for u in utts]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
    pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(dev)
    frames = int(np.ceil(args.seconds * 44100 / 512))
    from janus_amd.services.transcriber import TEMPERATURES
    pipe = JanusPipeline(args.model, max_length=args.max_length,
                         temperatures=TEMPERATURES if args.fallback else (0.0,))
    torch.cuda.synchronize()

    last = {}

    def step():
        if args.overlap > 0:
            # steady-state serving pipeline: batch i through mel / encoder / decoder / YIN,
            # batch i-1 through packets and the vocoder (the warm-up step primes it, so
            # every timed step carries a full encode and a full decode)
            enc, wav, pcm16 = pipe.step_overlapped(pcm, offs, lengths, frames, args.overlap)
        else:
            enc, wav, pcm16 = pipe.step(pcm, offs, lengths, frames)
        last["pcm16"] = pcm16
        return enc

    # overlapped: one priming step first (it fills the pipeline: encode only, no vocoder
    # pass), then the W warm-up steps, each a full encode + decode like the timed ones
    for _ in range(args.warmup + (1 if args.overlap > 0 else 0)):
        enc = step()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    pipe.vocoder.conv_stats(reset=True)
    pipe.vocoder.set_timing(True)
    times = []
    tok_counts = []
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_begin = time.perf_counter()
    for _ in range(args.steps):
        t0 = time.perf_counter()
        enc = step()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        tok_counts.append(enc.n_tokens)  # bookkeeping reduced after the timed region
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    t_end = time.perf_counter()
    pipe.vocoder.set_timing(False)
    tok_counts = [float(n.float().mean().item()) for n in tok_counts]
    fams = pipe.vocoder.family_stats(reset=False)
    flops, kms, launches = pipe.vocoder.conv_stats(reset=True)
    # latency of one batch through an IDLE pipeline (encode then decode back to back, nothing
    # else on the GPU), beside the serving figure (an utterance's encode step + decode step)
    idle = []
    if args.overlap > 0:
        pipe.flush(frames)
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pipe.step(pcm, offs, lengths, frames)
        torch.cuda.synchronize()
        idle.append(time.perf_counter() - t0)
    # whole-job time = max over ranks; result gather (packet bytes) once, outside the timing
    total_t = torch.tensor([t_end - t_begin], dtype=torch.float64, device=dev)
    n_packets = sum(p is not None for p in enc.packets)
    n_stats = int(enc.stats.shape[0]) if enc.stats is not None else 0
    if use_dist:
        dist.all_reduce(total_t, op=dist.ReduceOp.MAX)
        # result gather (RCCL over xGMI): the job's packets and per-utterance prosody
        # stats (rms, mean f0, voiced hops) on every rank, untimed
        pk_all, st_all = gather_results(enc.packets, enc.stats, dev)
        n_packets, n_stats = sum(p is not None for p in pk_all), int(st_all.shape[0])
    # host edges, outside the timed region (value has inputs resident in HBM): the PCM
    # upload of a batch and the download + RIFF framing of its int16 waveforms
    from janus_amd.vocoder import wav_bytes
    host_pcm = np.concatenate(utts + [np.zeros(1, np.float32)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _ = torch.from_numpy(host_pcm).to(dev)
    torch.cuda.synchronize()
    t_up = time.perf_counter() - t0
    t0 = time.perf_counter()
    if last.get("pcm16") is not None:
        h16 = last["pcm16"].cpu().numpy()
        _ = [wav_bytes(r) for r in h16]
    t_down = time.perf_counter() - t0
    wall = float(total_t.item())
    ms_per_step = wall / args.steps * 1000.0
    audio_s = world * B * args.seconds
    value = audio_s / (wall / args.steps)
    achieved = flops / (kms * 1e-3) / 1e12 if kms > 0 else 0.0
    n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
    cu_share = round(1.0 - args.overlap * 8 / n_cus, 4) if args.overlap > 0 else 1.0
    out = None
    if rank == 0:
        traffic = None
        try:
            tj = json.load(open(args.traffic_json))
            traffic = tj.get("bytes_per_launch")
        except Exception:
            traffic = None
        out = {
            "metric": "xRT (audio-s/wall-s) per GPU, 30s clips batch=64; p50 encode+decode latency",
            "value": round(value, 2),
            "unit": "xRT (audio-s/wall-s)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp16",
            "data": "synthetic (seeded source-filter speech, 48 kHz int16 grid; seeded synthetic weights)",
            "config": {"workload": "e2e encode+decode, Whisper base.en + Firefly-GAN vocoder, "
                                   f"{B} x {args.seconds:g} s utterances per GPU",
                       "model": args.model, "global_batch": world * B, "seq_len": 1500,
                       "parallelism": f"dp{world}", "max_length": args.max_length},
            "xrt_per_gpu": round(value / world, 2),
            # overlapped: an utterance is encoded in one step and vocoded in the next
            "p50_latency_ms": round(float(np.median(
                [a + b for a, b in zip(times[:-1], times[1:])] if args.overlap > 0 and len(times) > 1
                else times)) * 1000.0, 2),
            # one batch's encode + decode through an idle pipeline (sequential step), p50 of 3
            "p50_latency_idle_ms": round(float(np.median(idle)) * 1000.0, 2),
            "overlap": args.overlap,
            "step_ms": [round(t * 1000.0, 1) for t in times],
            "tokens_per_utt": round(float(np.mean(tok_counts)), 1),
            "packets_gathered": n_packets,
            # faster-whisper's gates on each T = 0 window; the fallback re-decodes run only
            # with --fallback (synthetic weights give avg_logprob far below -1, so every
            # window falls back)
            "gates": {"needs_fallback": int(sum(g[0] for g in enc.gates or [])),
                      "no_speech_skip": int(sum(g[1] for g in enc.gates or [])),
                      "mean_avg_logprob": round(float(np.mean([g[2] for g in enc.gates])), 3)
                      if enc.gates else None,
                      "fallback_run": bool(args.fallback),
                      "sampled_decodes": int(sum(g[6] for g in enc.gates or []))},
            "stats_gathered": n_stats,
            "host_edges_ms": {"pcm_upload": round(t_up * 1000.0, 1),
                              "wav_download_and_framing": round(t_down * 1000.0, 1)},
            "xrt_incl_host_edges": round(audio_s / (wall / args.steps + t_up + t_down), 2),
            "roofline": {
                "kernel": "conv1d implicit-GEMM (vocoder, v_mfma_f32_16x16x32_f16)",
                "bound": "mfma",
                "achieved": round(achieved, 2),
                "peak": MFMA_F16_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / MFMA_F16_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "launches": int(launches),
                "avg_launch_ms": round(kms / max(launches, 1), 4),
                "flops_per_launch": flops / max(launches, 1),
                # overlapped step: the conv launches own only the vocoder's CU share
                "cu_share": cu_share,
                "frac_of_cu_share": round(achieved / (MFMA_F16_PEAK_TFLOPS * cu_share), 4),
                # per family (fused-unit channel width; 0 = conv_pre + upsamplers): MFMA rate
                # and algorithmic HBM rate against their peaks on the CU share; "bound" =
                # the resource nearer its roofline (the narrow units are not MFMA-bound)
                "families": family_lines(fams, cu_share),
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args.model, float(np.mean(tok_counts)))
            except Exception as e:  # reported, never fatal to the bench line
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
