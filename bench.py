"""Janus hot-path benchmark: end-to-end encode + decode xRT on MI355X.

Workload (BASELINE.json metric "xRT (audio-s/wall-s) per GPU, 30s clips batch=64"):
per GPU, 64 seeded synthetic 30 s utterances at 48 kHz (janus_amd/workload.py) already
resident in HBM. One step = the whole batch through
  encode: log-mel([::3]) -> Whisper base.en encoder -> greedy decoder (<= 448 tokens,
          timestamp rules) over EVERY window of faster-whisper's seek loop
          (transcriber.py:53-57: the first 30 s window, then a window from the seek its
          last timestamp pair left, with the <|startofprev|> prompt) -> segments joined
          -> YIN + RMS prosody -> MessagePack packets
  decode: unpack -> "(emotion) text" prompt -> front end -> Firefly-GAN vocoder
          (30 s = 2584 latent frames -> 1 323 008 samples @ 44.1 kHz, f32 + int16)
Default (--stagger 1): the steady-state serving pipeline (JanusPipeline.step_staggered):
each step encodes batch i, runs ONE decoder call of 2 slot sets x 128 rows (a set takes
batch i's first windows together with an earlier batch's continuation windows; each set
advances 224 positions per call, a window completes in two calls) on 16 CUs of each XCD,
and renders the batch whose windows all settled on the other 16 (CU-masked streams);
every timed step takes in, decodes and renders 64 utterances' worth of windows (128 on
the synthetic weights). --stagger 0: the overlapped step; --overlap 0: back to back.
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
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r06.json"))
    ap.add_argument("--stagger", type=int, default=int(os.environ.get("JANUS_STAGGER", "1")),
                    help="1: continuous batching of windows in the decoder (JanusPipeline."
                         "step_staggered): each step's decoder calls advance 2 slot sets of 64 "
                         "rows; the first windows of batch i and the continuation windows of "
                         "the seek loop enter as fresh rows; 0: the overlapped step")
    ap.add_argument("--no-idle-latency", action="store_true",
                    help="skip the flush and the three idle-pipeline latency steps after the timed "
                         "region (profiling runs: only priming, warm-up and timed overlapped steps "
                         "then reach the kernel trace)")
    ap.add_argument("--config", type=int, default=4, choices=(1, 2, 3, 4, 5),
                    help="BASELINE.json config: 4 (default) = the headline, its per-GPU share "
                         "(64 x 30 s end to end); 1 = the 5 s WAV through the drop-in "
                         "Transcriber + prosody + packet; 2 = tiny.en + vocoder on one 30 s "
                         "utterance (latency); 3 = base.en encode-only, 64 x 30 s; 5 = "
                         "streaming duplex, --streams channels per GPU in real time")
    ap.add_argument("--streams", type=int, default=16,
                    help="config 5: capture channels per GPU (128 / 8)")
    ap.add_argument("--block-ms", type=int, default=320, help="config 5: block length")
    ap.add_argument("--stream-async", type=int, default=1,
                    help="config 5: 1 = encode + render on a worker stream while the next "
                         "blocks are ingested (StreamingEncoder(asynchronous=True))")
    ap.add_argument("--stream-t0", action="store_true",
                    help="config 5: decode at T = 0 only (default: faster-whisper's temperature "
                         "fallback, as the reference's transcribe_buffer runs it)")
    ap.add_argument("--duplex", type=int, default=1,
                    help="config 5: render every packet through the receiver's vocoder")
    ap.add_argument("--launch-check", action="store_true",
                    help="no GPU: spawn / join the ranks over gloo and print each rank's shard "
                         "(tests of the launcher)")
    ap.add_argument("--fallback-steps", type=int, default=3,
                    help="after the headline (T = 0) line, time this many steps of the same serving step with "
                         "faster-whisper's temperature fallback on and report them as "
                         "xrt_with_fallback (0: skip)")
    ap.add_argument("--first-window-steps", type=int, default=5,
                    help="after the headline, time this many steps decoding each clip's first "
                         "window only (the r05 serving semantics) and report xrt_first_window "
                         "(0: skip)")
    ap.add_argument("--fallback", action="store_true",
                    help="run faster-whisper's temperature fallback on windows failing their gates "
                         "(generate_with_fallback: 5 temperatures x best_of 5 sampled re-decodes); "
                         "off by default: the seeded synthetic weights fail every window (DESIGN.md §0)")
    return ap.parse_args()


def cpu_baseline(model: str, tokens_per_utt: float, seed: int = 999, windows: float = 1.0):
    """Oracle (CPU restatement) time for ONE whole 30 s utterance of the workload, every
    stage measured, nothing scaled: log-mel of the clip, the encoder on each of its seek
    windows (``windows`` per utterance on the GPU, rounded up), the sequential KV-cache
    greedy loop for as many tokens as the GPU emitted per utterance, split evenly over those
    windows (the reference's decode loop shape), YIN over all 30 s, and the vocoder for the
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
    x = synth_speech(seed, AUDIO_SECONDS)
    n_win = max(1, int(np.ceil(windows - 1e-6)))
    # tokens per window, at most what one 448-position window holds
    n_tok = max(1, min(int(round(tokens_per_utt / n_win)), 448 - len(tk.sot_sequence)))
    t = {}
    t0 = time.perf_counter()
    mel = ow.logmel(x, 3, jw.mel_filters())
    t["mel"] = time.perf_counter() - t0
    t["encoder"] = t["decoder"] = 0.0
    n_dec = 0
    for _ in range(n_win):   # every window costs one encoder pass and one decode loop
        t0 = time.perf_counter()
        enc = ow.encoder(mel[None], W, cfg)
        t["encoder"] += time.perf_counter() - t0
        t0 = time.perf_counter()
        dec = ow.greedy_cached(enc.half().float(), W, cfg, tk, max_length=len(tk.sot_sequence) + n_tok)
        t["decoder"] += time.perf_counter() - t0
        n_dec += len(dec[0]["tokens"])
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
                   f"every stage measured: mel, encoder on each of {n_win} window(s), sequential "
                   f"KV-cache greedy loop over {n_dec} tokens, YIN over 30 s (1 thread), vocoder 30 s "
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


def decoder_bytes(cfg, B, positions):
    """Algorithmic HBM bytes the greedy decoder must move per position, at
    batch B over `positions` steps (position p attends over p + 1 keys):
      cross_attention  the encoder output, read once per layer (absorbed projections):
                       L * B * Te * d * 2
      self_attention   the K and V cache rows that exist, averaged over the positions:
                       L * B * (positions + 1) / 2 * d * 2 * 2
      layer_weights    per layer QKV 3d^2, O d^2, absorbed query H d^2, per-head value d^2,
                       cross O d^2, fc1 4d^2, fc2 4d^2 (fp16): L * (14 + H) * d^2 * 2
      vocab_projection the tied token embedding: V * d * 2
    Activations (a few hundred KB per launch) are left out."""
    d, H, L, Te, V = cfg.d_model, cfg.n_heads, cfg.dec_layers, cfg.n_audio_ctx, cfg.n_vocab
    return {"cross_attention": L * B * Te * d * 2,
            "self_attention": L * B * (positions + 1) / 2.0 * d * 2 * 2,
            "layer_weights": L * (14 + H) * d * d * 2,
            "vocab_projection": V * d * 2}


def decoder_roofline(cfg, B, positions, launches, side_ms, cu_share, tkv_positions=None):
    """roofline.decoder: the side that sets the overlapped step. side_ms = decoder-side
    wall time per step (HIP events on the decoder's CU-masked stream, timed region) over
    `positions` decoder steps of B rows; tkv_positions: the decode length whose average key
    count the rows see (staggered: the two row sets together see a full decode's)."""
    if not side_ms or positions <= 0:
        return None
    by = decoder_bytes(cfg, B, tkv_positions or positions)
    per_pos = sum(by.values())
    us = side_ms * 1000.0 / positions
    gbs = per_pos / (us * 1e-6) / 1e9
    return {"kernel": "greedy decoder, one position (cross-attention, self-attention, "
                      "projections, vocabulary projection + selection)",
            "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "cu_share": cu_share,
            "frac_of_cu_share": round(gbs / (HBM_PEAK_GBS * cu_share), 4),
            "bytes_per_position": int(per_pos),
            "bytes_breakdown": {k: int(v) for k, v in by.items()},
            "rows": B, "positions": positions, "side_ms": round(side_ms, 2),
            "us_per_position": round(us, 2),
            "launches_per_position": round(launches / positions, 2) if launches else None,
            "us_per_launch": round(us * positions / launches, 2) if launches else None}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _line(args, metric, value, unit, ms, config, **extra):
    out = {"metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
           "higher_is_better": True, "scaling": "none (single GPU config)", "vs_baseline": None,
           "dtype": "fp16",
           "data": "synthetic (seeded source-filter speech; seeded synthetic weights)",
           "config": config}
    out.update(extra)
    print(json.dumps(out), flush=True)


def _timed(fn, steps, warmup):
    """fn() once per step, host-synchronised, after `warmup` untimed calls: per-step
    seconds."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(steps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    return t


def run_config1(args):
    """BASELINE config 1: one 5 s 16 kHz mono WAV through the drop-in Transcriber
    (transcriber.py:66-91, tiny.en) + ProsodyExtractor (prosody.py:45-104, on the 48 kHz
    buffer whose [::3] is the WAV) + JanusPacket.serialize (protocol.py:57-121): the
    reference's CPU plumbing path, here on the GPU; per-call latency and xRT."""
    import tempfile
    import wave
    from janus_amd.common.protocol import JanusMode, JanusPacket
    from janus_amd.services.prosody import ProsodyExtractor
    from janus_amd.services.transcriber import Transcriber
    from janus_amd.workload import synth_speech
    secs = 5.0
    x = synth_speech(1000, secs, sr=16000)
    path = os.path.join(tempfile.mkdtemp(), "config1.wav")
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes((x * 32768).astype("<i2").tobytes())
    tr = Transcriber("tiny.en")
    if not args.fallback:   # the headline's setting (T = 0); --fallback: faster-whisper's default
        import functools
        tr.model.transcribe = functools.partial(tr.model.transcribe, temperature=0.0)
    ex = ProsodyExtractor(48000)
    buf48 = np.repeat(x, 3)
    res = {}

    def one():
        text = tr.transcribe_file(path)
        tags = ex.analyze_buffer(buf48)
        res["packet"] = JanusPacket(text, JanusMode.SEMANTIC_VOICE, tags, "Auto", 1.0).serialize()
        res["text"] = text
    t = _timed(one, args.steps, args.warmup)
    p50 = float(np.median(t))
    cpu = None
    if not args.no_cpu_baseline:
        try:
            cpu = cpu_config1(x, buf48, args.fallback)
            cpu["packet_equal"] = cpu.pop("packet") == res["packet"]
        except Exception as e:
            cpu = {"error": repr(e)}
    _line(args, "config 1: 5 s WAV -> tiny.en STT + prosody + MessagePack, latency", secs / p50,
          "xRT (audio-s/wall-s)", p50 * 1000.0,
          {"workload": "5 s 16 kHz WAV through Transcriber('tiny.en').transcribe_file + "
                       "ProsodyExtractor + JanusPacket.serialize", "model": "tiny.en",
           "global_batch": 1, "fallback": bool(args.fallback)},
          p50_latency_ms=round(p50 * 1000.0, 2), step_ms=[round(v * 1000.0, 2) for v in t],
          packet_bytes=len(res["packet"]), roofline=None,
          roofline_note="latency-bound single-utterance plumbing: no kernel near a roofline",
          cpu_baseline=cpu)


def cpu_config1(x16, buf48, fallback):
    """Config 1 on the CPU oracle, the whole job (the reference's own path is CPU): the
    seek loop (oracle.whisper.transcribe_segments, T = 0 unless --fallback) on the WAV's
    int16 samples, the stateful prosody oracle on the 48 kHz buffer, the oracle packer."""
    from janus_amd import whisper as jw
    from janus_amd.tokenizer import load_tokenizer
    from oracle import packet as opk
    from oracle import whisper as ow
    from oracle.prosody import OracleProsody
    affinity = len(os.sched_getaffinity(0))
    threads = min(affinity, int(os.environ.get("OMP_NUM_THREADS", affinity)))
    torch.set_num_threads(threads)
    cfg = jw.CONFIGS["tiny.en"]
    W = jw.synthetic_weights(cfg, 0)
    tk = load_tokenizer()
    a = (x16 * 32768).astype("<i2").astype(np.float32) / 32768.0
    temps = (0.0, 0.2, 0.4, 0.6, 0.8, 1.0) if fallback else (0.0,)
    t0 = time.perf_counter()
    segs, _ = ow.transcribe_segments(a, W, cfg, tk, jw.mel_filters(), temperatures=temps)
    text = " ".join(sg[2].strip() for sg in segs).strip()
    tags = OracleProsody(48000).analyze_buffer(buf48)[0]
    pk = opk.serialize(text, 0, tags, "Auto", 1.0)
    dt = time.perf_counter() - t0
    return {"value": (len(x16) / 16000.0) / dt, "unit": "xRT (audio-s/wall-s)", "cores": threads,
            "kind": "port", "latency_ms": round(dt * 1000.0, 1), "packet": pk,
            "sample": "the whole config-1 job on the oracle: seek loop + prosody + packer",
            "cpu_model": _cpu_model()}


def run_config2(args):
    """BASELINE config 2: tiny.en encode (mel, encoder, greedy decoder, YIN, packet) + the
    Firefly-GAN decode of the packet, ONE 30 s utterance, back to back on the whole GPU
    (JanusPipeline.step); p50 latency over the timed steps, xRT = 30 s / p50."""
    from janus_amd.pipeline import JanusPipeline
    from janus_amd.services.transcriber import TEMPERATURES
    from janus_amd.workload import synth_speech
    dev = torch.device("cuda", 0)
    x = synth_speech(2000, args.seconds)
    offs = torch.tensor([0, len(x)], dtype=torch.int64, device=dev)
    pcm = torch.from_numpy(np.concatenate([x, np.zeros(1, np.float32)])).to(dev)
    frames = int(np.ceil(args.seconds * 44100 / 512))
    pipe = JanusPipeline("tiny.en", max_length=args.max_length,
                         temperatures=TEMPERATURES if args.fallback else (0.0,))
    last = {}

    def one():
        last["r"] = pipe.step(pcm, offs, [len(x)], frames)
    for _ in range(args.warmup):
        one()
    torch.cuda.synchronize()
    pipe.vocoder.conv_stats(reset=True)
    pipe.vocoder.family_stats(reset=True)
    pipe.vocoder.set_timing(True)
    t = _timed(one, args.steps, 0)
    pipe.vocoder.set_timing(False)
    fams = pipe.vocoder.family_stats(reset=False)
    flops, kms, launches = pipe.vocoder.conv_stats(reset=True)
    p50 = float(np.median(t))
    ach = flops / (kms * 1e-3) / 1e12 if kms > 0 else 0.0
    enc = last["r"][0]
    cpu = None
    if not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline("tiny.en", float(enc.n_tokens.float().mean().item()), seed=2000)
        except Exception as e:
            cpu = {"error": repr(e)}
    _line(args, "config 2: tiny.en encode + Firefly-GAN decode, one 30 s utterance, p50 latency",
          args.seconds / p50, "xRT (audio-s/wall-s)", p50 * 1000.0,
          {"workload": f"1 x {args.seconds:g} s utterance: mel, tiny.en encoder, greedy decoder "
                       "(<= 448 tokens), YIN, packet, then unpack, prompt, vocoder "
                       f"({frames} frames)", "model": "tiny.en", "global_batch": 1,
           "max_length": args.max_length, "fallback": bool(args.fallback)},
          p50_latency_ms=round(p50 * 1000.0, 2), step_ms=[round(v * 1000.0, 2) for v in t],
          tokens=int(enc.n_tokens[0].item()),
          roofline={"kernel": "vocoder conv / fused ResBlock1 units (whole GPU, batch 1)",
                    "bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_F16_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / MFMA_F16_PEAK_TFLOPS, 4),
                    "traffic": None, "launches": int(launches),
                    "avg_launch_ms": round(kms / max(launches, 1), 4),
                    "families": family_lines(fams, 1.0)},
          cpu_baseline=cpu)


def encoder_flops(cfg, B):
    """Algorithmic FLOPs of one encoder forward at batch B (30 s windows): conv1 (k3, 80 ->
    d, 3000 frames) + conv2 (k3 stride 2, d -> d, 1500 frames), and per layer the
    projections 24 T d^2 plus attention 4 T^2 d."""
    d, T, L = cfg.d_model, cfg.n_audio_ctx, cfg.enc_layers
    stem = 2 * 3 * (2 * T) * 80 * d + 2 * 3 * T * d * d
    gemm = L * 24 * T * d * d
    attn = L * 4 * T * T * d
    return {"stem": B * stem, "projections": B * gemm, "attention": B * attn}


def run_config3(args):
    """BASELINE config 3: base.en encode-only (log-mel + encoder: conv stem, 6 layers of
    MFMA attention / FFN) on 64 x 30 s utterances; xRT and the encoder's MFMA fraction,
    plus per-kernel lines for the projection GEMM (gemm_big) and the attention kernel at
    the same shapes (HIP events)."""
    import math
    from janus_amd import _native as nat
    from janus_amd.whisper import CONFIGS, WhisperEngine
    from janus_amd.workload import synth_speech
    dev = torch.device("cuda", 0)
    B = args.batch
    cfg = CONFIGS[args.model]
    utts = [synth_speech(3000 + i, args.seconds) for i in range(B)]
    lengths = [len(u) for u in utts]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
    pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(dev)
    w = WhisperEngine(cfg, seed=0)

    def one():
        return w.encode(w.logmel(pcm, offs, B, 3))
    for _ in range(args.warmup):
        one()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    mel_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    t = []
    for i in range(args.steps):
        t0 = time.perf_counter()
        mel_ev[i][0].record()
        mel = w.logmel(pcm, offs, B, 3)
        mel_ev[i][1].record()
        ev[i][0].record()
        w.encode(mel)
        ev[i][1].record()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    enc_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    mel_ms = float(np.mean([a.elapsed_time(b) for a, b in mel_ev]))
    fl = encoder_flops(cfg, B)
    tot = sum(fl.values())
    ach = tot / (enc_ms * 1e-3) / 1e12
    # the encoder's kernels at the same shapes, alone (kernel ABI, HIP events)
    s = torch.cuda.current_stream().cuda_stream
    M, d = B * cfg.n_audio_ctx, cfg.d_model
    kern = []
    g = torch.Generator(device=dev).manual_seed(1)
    for name, N, K, epi in [("qkv", 3 * d, d, 0), ("o_resid", d, d, 2), ("fc1_gelu", 4 * d, d, 1),
                            ("fc2_resid", d, 4 * d, 2)]:
        A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).half()
        Wm = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) / math.sqrt(K)).half()
        bias = torch.randn(N, device=dev, generator=g)
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if epi == 2 else torch.float16)

        def run():
            nat.call("janus_gemm_f16", epi, A.data_ptr(), K, Wm.data_ptr(), K, bias.data_ptr(),
                     C.data_ptr(), N, C.data_ptr() if epi == 2 else None, N, M, N, K, s)
        run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 100.0
        tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        kern.append({"kernel": f"gemm_big {name} ({M}x{N}x{K})", "us": round(us, 1),
                     "achieved_tflops": round(tf, 1), "frac": round(tf / MFMA_F16_PEAK_TFLOPS, 4)})
        del A, Wm, C
    qkv = (torch.randn(B, cfg.n_audio_ctx, 3 * d, device=dev, generator=g) * 1.5).half()
    out = torch.empty(B, cfg.n_audio_ctx, d, dtype=torch.float16, device=dev)
    run = lambda: nat.call("janus_attention_f16", qkv.data_ptr(), out.data_ptr(), B,
                           cfg.n_audio_ctx, cfg.n_heads, 0.125, s)
    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 100.0
    tf = 4.0 * B * cfg.n_heads * cfg.n_audio_ctx ** 2 * 64 / (us * 1e-6) / 1e12
    kern.append({"kernel": f"attention_st ({B} x {cfg.n_heads} heads x {cfg.n_audio_ctx}^2)",
                 "us": round(us, 1), "achieved_tflops": round(tf, 1),
                 "frac": round(tf / MFMA_F16_PEAK_TFLOPS, 4)})
    step_s = (mel_ms + enc_ms) / 1000.0
    cpu = None
    if not args.no_cpu_baseline:
        try:
            cpu = cpu_encoder_baseline(args.model)
        except Exception as e:
            cpu = {"error": repr(e)}
    _line(args, "config 3: base.en encode-only, batch 64 x 30 s, xRT and MFMA fraction",
          B * args.seconds / step_s, "xRT (audio-s/wall-s)", step_s * 1000.0,
          {"workload": f"log-mel + {args.model} encoder, {B} x {args.seconds:g} s", "model": args.model,
           "global_batch": B, "seq_len": cfg.n_audio_ctx},
          mel_ms=round(mel_ms, 3), encoder_ms=round(enc_ms, 3),
          host_step_ms=[round(v * 1000.0, 2) for v in t],
          roofline={"kernel": "Whisper encoder forward (stem conv, QKV/O/fc1/fc2 on gemm_big, "
                              "attention_st), HIP events around the encoder",
                    "bound": "mfma", "achieved": round(ach, 1), "peak": MFMA_F16_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / MFMA_F16_PEAK_TFLOPS, 4),
                    "traffic": None, "flops": {k: float(v) for k, v in fl.items()},
                    "kernels": kern},
          cpu_baseline=cpu)


def cpu_encoder_baseline(model):
    """Oracle log-mel + encoder for ONE 30 s utterance (numpy / torch fp32)."""
    from janus_amd import whisper as jw
    from janus_amd.workload import synth_speech
    from oracle import whisper as ow
    affinity = len(os.sched_getaffinity(0))
    threads = min(affinity, int(os.environ.get("OMP_NUM_THREADS", affinity)))
    torch.set_num_threads(threads)
    cfg = jw.CONFIGS[model]
    W = jw.synthetic_weights(cfg, 0)
    x = synth_speech(3999, AUDIO_SECONDS)
    t0 = time.perf_counter()
    mel = ow.logmel(x, 3, jw.mel_filters())
    ow.encoder(mel[None], W, cfg)
    dt = time.perf_counter() - t0
    return {"value": AUDIO_SECONDS / dt, "unit": "xRT (audio-s/wall-s)", "cores": threads,
            "kind": "port", "sample": "oracle log-mel + fp32 encoder, one 30 s utterance",
            "cpu_model": _cpu_model()}


def run_config5(args, rank, world, use_dist, dev):
    """BASELINE config 5: 16 concurrent 48 kHz capture channels per GPU (128 over 8 GPUs)
    arriving in real time as 320 ms blocks (10 x 1536-sample chunks); channel s on rank
    s mod N. Per block every chunk is gated and phrases are segmented per channel
    (engine.py:438-506); completed phrases are encoded as one GPU batch (Whisper + YIN with
    per-channel detector state + packet, engine.py:510-552) on a worker stream and, in
    duplex mode, rendered by the receiver leg (engine.py:220-286: prompt -> vocoder at the
    phrase's duration). After the run every rank's per-block push latencies and
    per-phrase duplex latencies (phrase complete -> packet + rendered audio) are
    all-gathered (RCCL), so rank 0 reports the node's p50 / p99 and whether every block
    and phrase stayed inside the 320 ms block. Two legs, the same channels: faster-whisper's
    temperature fallback (the reference's transcribe_buffer, engine.py:510-527: the line's
    value) and T = 0 alone (``t0``); --stream-t0 runs the T = 0 leg only."""
    from janus_amd.services.transcriber import TEMPERATURES
    legs = [("t0", (0.0,))] if args.stream_t0 else [("fallback", TEMPERATURES), ("t0", (0.0,))]
    res = {name: _stream_leg(args, rank, world, use_dist, dev, temps) for name, temps in legs}
    if rank != 0:
        return
    main_leg = res[legs[0][0]]
    out = {"metric": "config 5: streaming duplex, 16 kHz channels x 320 ms chunks, per-phrase "
                     "encode+decode p50 latency (phrase complete -> packet + rendered audio)",
           "value": main_leg["phrase_p50_ms"], "unit": "ms", "n_gpus": world,
           "steps": main_leg["blocks"], "warmup": 4, "ms_per_step": main_leg["p50_ms"],
           "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "fp16",
           "data": "synthetic seeded speech phrases with silences per channel; energy speech "
                   "gate; seeded synthetic weights",
           "config": {"workload": f"{args.streams * world} channels ({args.streams} per GPU, channel s "
                                  f"on rank s mod {world}), {args.seconds:g} s of {args.block_ms} ms "
                                  "blocks in real time", "model": args.model,
                      "streams_total": args.streams * world, "parallelism": f"dp{world}",
                      "max_length": args.max_length},
           "streams_total": args.streams * world, "streams_per_gpu": args.streams,
           "block_ms": args.block_ms, "asynchronous": bool(args.stream_async),
           "duplex": bool(args.duplex), "leg": legs[0][0]}
    out.update(main_leg)
    if len(legs) > 1:
        out["t0"] = res["t0"]
    out["roofline"] = None
    out["roofline_note"] = ("real-time arrival: per-phrase batches of a few 1.5-6 s phrases, "
                            "latency-bound; the kernels' rooflines are the config-4 line's")
    out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)


def _stream_leg(args, rank, world, use_dist, dev, temps):
    """One config-5 run at the temperatures ``temps``: per-block push and per-phrase duplex
    latencies gathered over the ranks (rank 0's dict; None elsewhere)."""
    from janus_amd.streaming import CHUNK, StreamingEncoder
    from janus_amd.whisper import CONFIGS, WhisperEngine
    from janus_amd.workload import channel_audio, synth_speech
    per_block = int(round(args.block_ms / 32.0))          # 1536 samples = 32 ms
    n_blocks = int(args.seconds * 1000 / args.block_ms)
    total = n_blocks * per_block * CHUNK
    n_total = args.streams * world
    mine = [s for s in range(n_total) if s % world == rank]
    audio = np.stack([channel_audio(s, total) for s in mine])
    S = len(mine)
    w = WhisperEngine(CONFIGS[args.model], seed=0)
    rx = None
    if args.duplex:
        from janus_amd.pipeline import PacketRenderer
        rx = PacketRenderer()   # the far end's vocoder alone (no second Whisper engine)
    enc = StreamingEncoder(S, w, max_length=args.max_length, asynchronous=bool(args.stream_async),
                           receiver=rx, temperatures=temps)
    # warm-up: one block of speech + silence on a scratch encoder (graph capture, allocations)
    warm = StreamingEncoder(S, w, max_length=args.max_length, receiver=rx, temperatures=temps)
    z = np.zeros((S, per_block * CHUNK), np.float32)
    sp = np.tile(synth_speech(1, per_block * CHUNK / 48000.0)[None, :per_block * CHUNK], (S, 1))
    warm.push(sp)
    for _ in range(3):
        warm.push(z)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    phrases = 0
    t_start = time.perf_counter()
    for b in range(n_blocks):
        # blocks arrive in real time: block b is complete at t_start + (b + 1) * block
        wait = t_start + (b + 1) * args.block_ms / 1000.0 - time.perf_counter()
        if wait > 0:
            time.sleep(wait)
        out = enc.push(audio[:, b * per_block * CHUNK:(b + 1) * per_block * CHUNK])
        phrases += len(out)
    phrases += len(enc.flush())
    t_total = time.perf_counter() - t_start
    enc.close()
    warm.close()
    lat, plat = list(enc.latencies), list(enc.phrase_latencies)
    counts = [phrases, enc.max_queue, enc.extra_windows, getattr(enc, "worker_batches", 0)]
    if use_dist:
        from janus_amd.dist import gather_values
        lat, plat = gather_values(lat, dev), gather_values(plat, dev)
        per_rank = gather_values(counts, dev)
        counts = [sum(per_rank[0::4]), max(per_rank[1::4]), sum(per_rank[2::4]), sum(per_rank[3::4])]
        wall = torch.tensor([t_total], dtype=torch.float64, device=dev)
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
        t_total = float(wall.item())
    if rank != 0:
        return None
    lat = np.array(lat) * 1000.0
    plat = np.array(plat) * 1000.0 if len(plat) else np.zeros(1)
    p50, p99 = float(np.percentile(lat, 50)), float(np.percentile(lat, 99))
    pp50, pp99 = float(np.percentile(plat, 50)), float(np.percentile(plat, 99))
    return {"temperatures": list(temps), "fallback": len(temps) > 1, "blocks": n_blocks,
            "phrases": int(counts[0]),
            # per-block push latency (gate + segmentation of every channel's 320 ms block)
            "p50_ms": round(p50, 2), "p99_ms": round(p99, 2), "max_ms": round(float(lat.max()), 2),
            # per-phrase duplex latency (phrase complete -> packet + rendered audio)
            "phrase_p50_ms": round(pp50, 2), "phrase_p99_ms": round(pp99, 2),
            "phrase_max_ms": round(float(plat.max()), 2),
            "worker_max_queue": int(counts[1]),
            # worker batches (jobs queued while one ran are merged into the next batch)
            "worker_batches": int(counts[3]), "wall_s": round(t_total, 2),
            "audio_s": round(n_blocks * args.block_ms / 1000.0, 2),
            "realtime": bool(p99 < args.block_ms and pp99 < args.block_ms),
            # the worker kept up: every phrase encoded + rendered before the stream ended plus
            # one block, queue bounded
            "kept_up": bool(t_total < n_blocks * args.block_ms / 1000.0 + args.block_ms / 1000.0 * 2),
            "extra_seek_windows": int(counts[2])}


def run_launch_check(args, rank, world):
    """--launch-check: the multi-process plumbing without a GPU (gloo): every rank reports
    (rank, world, its utterance shard of world x batch, its config-5 channels) and rank 0
    prints them gathered, one JSON line. tests/test_distributed.py drives it through
    ``bench.py --gpus 2`` (the spawning launcher) on the CPU."""
    from janus_amd.dist import gather_values, shard
    if world > 1:
        dist.init_process_group("gloo")
    u0, u1 = shard(rank, world, world * args.batch)
    chans = [s for s in range(args.streams * world) if s % world == rank]
    mine = [rank, world, u0, u1, len(chans), chans[0] if chans else -1]
    allv = gather_values(mine, torch.device("cpu")) if world > 1 else mine
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        ranks = [allv[i:i + 6] for i in range(0, len(allv), 6)]
        print(json.dumps({"launch_check": True, "world": world,
                          "ranks": [{"rank": int(r[0]), "world": int(r[1]),
                                     "shard": [int(r[2]), int(r[3])], "channels": int(r[4]),
                                     "first_channel": int(r[5])} for r in ranks],
                          "pid": os.getpid()}), flush=True)


def main():
    args = parse()
    from janus_amd import launch
    launched = os.environ.get("WORLD_SIZE") is not None
    if args.config in (1, 2, 3) and args.gpus != 1:
        print(f"bench.py: config {args.config} is a single-GPU configuration (--gpus 1)",
              file=sys.stderr)
        sys.exit(2)
    # --gpus N without a launcher: N fresh rank processes of this script, started before
    # this process makes any HIP call; with a launcher, --gpus must match WORLD_SIZE
    err = None if args.launch_check else launch.check_world(args.gpus)
    if err is not None:
        print(f"bench.py: {err}", file=sys.stderr, flush=True)
        sys.exit(2)
    if not launched and args.gpus > 1:
        sys.exit(launch.spawn(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        run_launch_check(args, rank, world)
        return
    if args.config in (1, 2, 3):
        torch.cuda.set_device(0)
        {1: run_config1, 2: run_config2, 3: run_config3}[args.config](args)
        return
    torch.cuda.set_device(local)
    # JANUS_DIST_FORCE=1: the RCCL path (process group, barriers, max-over-ranks all-reduce,
    # result gather) at world size 1 too — exercises it on a one-GPU box
    use_dist = world > 1 or os.environ.get("JANUS_DIST_FORCE") == "1"
    if use_dist:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.config == 5:
        run_config5(args, rank, world, use_dist, torch.device("cuda", local))
        if use_dist:
            dist.barrier()
            dist.destroy_process_group()
        return

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
    from janus_amd.pipeline import ServingTuning
    # the measured serving geometry; JANUS_<FIELD> overrides one field for an A/B
    tuning = ServingTuning.from_env()
    pipe = JanusPipeline(args.model, max_length=args.max_length,
                         temperatures=TEMPERATURES if args.fallback else (0.0,), tuning=tuning)
    torch.cuda.synchronize()

    last = {}

    def step():
        if args.overlap > 0 and args.stagger:
            # continuous batching of windows: batch i's first windows and the queued
            # continuation windows of earlier batches in the decoder calls, the vocoder of the
            # oldest finished batch beside them (with the fallback on, the completed windows
            # that fail their gates re-decode first, on the whole GPU)
            enc, wav, pcm16 = pipe.step_staggered(pcm, offs, lengths, frames, args.overlap)
        elif args.overlap > 0:
            # steady-state serving pipeline: batch i through mel / encoder / decoder / YIN,
            # batch i-1 through packets and the vocoder (the warm-up step primes it, so
            # every timed step carries a full encode and a full decode)
            enc, wav, pcm16 = pipe.step_overlapped(pcm, offs, lengths, frames, args.overlap)
        else:
            enc, wav, pcm16 = pipe.step(pcm, offs, lengths, frames)
        last["pcm16"] = pcm16
        return enc

    # priming: the pipeline's depth in steps (staggered: until the first batch comes out,
    # 3 steps with two windows per clip), then the W warm-up steps, each a full step like
    # the timed ones
    sets = max(2, tuning.stagger_sets) if args.stagger else 1
    calls = tuning.calls() if args.stagger else 1
    depth = (pipe.staggered_depth() if args.stagger else 1) if args.overlap > 0 else 0
    enc = None
    for _ in range(depth):
        enc = step()
    guard = 0
    while args.overlap > 0 and enc is None and guard < 8:   # longer seek loops fill later
        enc = step()
        guard += 1
    for _ in range(args.warmup):
        enc = step()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    pipe.vocoder.conv_stats(reset=True)
    pipe.vocoder.set_timing(True)
    pipe.side_events = [] if args.overlap > 0 else None
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
        tok_counts.append(enc)  # bookkeeping reduced after the timed region
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    t_end = time.perf_counter()
    pipe.vocoder.set_timing(False)
    yin_dec_utts = (getattr(pipe, "_stag", None) or {}).get("n_dec") if args.stagger == 1 else None
    # rows per decoder call: every slot set's R rows (R = 2B with all windows)
    dec_rows = sets * ((getattr(pipe, "_stag", None) or {}).get("R", B) if args.stagger else B)
    sides = [(e[0].elapsed_time(e[1]), e[2].elapsed_time(e[3])) for e in (pipe.side_events or [])]
    pipe.side_events = None
    dec_positions, dec_launches = pipe.whisper.decode_info()
    # tokens sampled per utterance over all of its windows, and the windows themselves
    tok_counts = [float(np.mean(e.sampled)) for e in tok_counts]
    windows = [int(x) for x in enc.windows]
    fams = pipe.vocoder.family_stats(reset=False)
    flops, kms, launches = pipe.vocoder.conv_stats(reset=True)
    # faster-whisper's seek loop decodes windows until every clip's seek has reached its
    # content: clips of the last timed batch left short of it (0 when every window was decoded)
    content = [(n + 2) // 3 // 160 for n in lengths]
    seek_extra = int(sum(1 for st, c in zip(enc.streams, content) if st.seek < c))
    flush = {0: pipe.flush, 1: pipe.flush_staggered}

    def timed_leg(n_steps, prime):
        """n_steps timed steps of the current setting after `prime` untimed ones (the
        pipeline's depth plus a warm step), then drained: (per-step seconds, last result)."""
        r = None
        for _ in range(prime):
            r = step() or r
        ts = []
        for _ in range(n_steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = step() or r
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        flush[min(args.stagger, 1)](frames)
        return ts, r
    # latency of one batch through an IDLE pipeline (encode then decode back to back, nothing
    # else on the GPU), beside the serving figure (an utterance's encode step + decode step)
    idle = []
    if args.overlap > 0 and not args.no_idle_latency:
        flush[args.stagger](frames)
    for _ in range(0 if args.no_idle_latency else 3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pipe.step(pcm, offs, lengths, frames)
        torch.cuda.synchronize()
        idle.append(time.perf_counter() - t0)
    # the latency operating point: the overlapped step (--stagger 0: an utterance's encode +
    # decode step, then its vocoder step) timed right after, beside the staggered headline
    # (four steps per utterance with two windows each): p50 of consecutive step pairs
    ov = None
    if args.overlap > 0 and args.stagger != 0 and not args.no_idle_latency and not args.fallback:
        ov_t = []
        for i in range(2 + 5):   # priming + warm-up, then 5 timed
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pipe.step_overlapped(pcm, offs, lengths, frames, args.overlap)
            torch.cuda.synchronize()
            if i >= 2:
                ov_t.append(time.perf_counter() - t0)
        pipe.flush(frames)
        ov = {"p50_latency_ms": round(float(np.median([ov_t[i] + ov_t[i + 1]
                                                        for i in range(len(ov_t) - 1)])) * 1000.0, 2),
              "step_ms": [round(v * 1000.0, 1) for v in ov_t],
              "xrt": round(B * args.seconds / float(np.mean(ov_t)), 2)}
    # the r05 serving semantics beside the headline: each clip's FIRST window only (the seek
    # loop stopped after it), the same staggered step with one decoder call per step
    fw = None
    if (args.overlap > 0 and args.stagger == 1 and pipe.tuning.all_windows
            and not args.no_idle_latency and args.first_window_steps > 0):
        pipe.tuning.all_windows = False
        fw_t, fwr = timed_leg(args.first_window_steps, pipe.staggered_depth() + 1)
        pipe.tuning.all_windows = True
        fw = {"xrt": round(B * args.seconds / float(np.mean(fw_t)), 2),
              "step_ms": [round(v * 1000.0, 1) for v in fw_t],
              "windows_decoded": int(sum(fwr.windows)) if fwr is not None else None}
    # the same serving step with faster-whisper's temperature fallback on (the library
    # default; every window of the seeded synthetic model fails its gates, so each runs all
    # five sampled temperatures x best_of 5), every window of the seek loop: reported beside
    # the T = 0 headline
    fb = None
    if (args.fallback_steps > 0 and not args.fallback and not args.no_idle_latency
            and args.overlap > 0):
        pipe.temperatures = TEMPERATURES
        fb_t, fenc = timed_leg(args.fallback_steps, depth + 1)
        pipe.temperatures = (0.0,)
        fb = {"xrt": round(B * args.seconds / float(np.mean(fb_t)), 2),
              "step": {0: "overlapped", 1: "staggered"}[args.stagger],
              "step_ms": [round(v * 1000.0, 1) for v in fb_t],
              "windows_decoded": int(sum(fenc.windows)) if fenc is not None else None,
              "sampled_decodes": int(sum(s.fallback_decodes for s in fenc.streams)) if fenc else None,
              "windows_failing_t0": int(sum(s.fallbacks for s in fenc.streams)) if fenc else None}
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
            # measured on a standalone forward of tj["batch"] utterances; the line's launches
            # are the main vocoder context's, which renders B minus the utterances the
            # staggered step hands to the decoder's CUs: bytes scale with the utterances
            main_b = B - int(getattr(pipe, "voc_dec_utts", 0) or 0)
            traffic = tj.get("bytes_per_launch") * main_b / float(tj.get("batch", 64))
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
            # an utterance's steps: encode + decode, then vocoder (overlapped: 2 steps);
            # staggered with two windows per clip: first window (one step), continuation
            # window (two steps), then the vocoder (4 steps)
            # (fewer timed steps than the depth: depth + 1 median steps)
            "p50_latency_ms": round(float(
                np.median([sum(times[i:i + depth + 1]) for i in range(len(times) - depth)])
                if args.overlap > 0 and len(times) > depth
                else (depth + 1 if args.overlap > 0 else 1) * np.median(times)) * 1000.0, 2),
            # the latency operating point: the overlapped step (--stagger 0), timed after the
            # headline on the same pipeline (an utterance's encode + decode step, then its
            # vocoder step); the staggered headline trades one more step of latency for xRT
            "p50_latency_ms_overlapped": ov["p50_latency_ms"] if ov else None,
            "overlapped": ov,
            "stagger": int(args.stagger),
            "stagger_sets": sets if args.stagger else None,
            # the headline decodes at T = 0 only (faster-whisper's fallback temperatures are
            # the xrt_with_fallback leg below, or --fallback)
            "temperatures": list(pipe.temperatures) if args.fallback else [0.0],
            # one batch's encode + decode through an idle pipeline (sequential step), p50 of 3
            "p50_latency_idle_ms": round(float(np.median(idle)) * 1000.0, 2) if idle else None,
            # wall time of the two CU partitions per timed step (HIP events on each side's
            # stream): vocoder + YIN, greedy decoder
            "side_ms": {"vocoder": [round(a, 1) for a, _ in sides],
                        "decoder": [round(b, 1) for _, b in sides]} if sides else None,
            "decoder_calls_per_step": calls if args.stagger else 1,
            # staggered step: utterances whose YIN ran on the decoder side in the last timed
            # step (self-balancing split, JanusPipeline._yin_split)
            "yin_dec_utts": yin_dec_utts,
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
            # faster-whisper's seek loop over every clip (transcriber.py:53-57): the windows
            # the last timed batch decoded (a first window per clip, then one from the seek
            # its last timestamp pair left), and clips left short of their content (0)
            "all_windows": bool(pipe.tuning.all_windows),
            "windows_decoded": int(sum(windows)),
            "windows_per_utt": round(float(np.mean(windows)), 3),
            "seek_windows_extra": seek_extra,
            # the same staggered step decoding each clip's FIRST window only (the r05 serving
            # semantics, one decoder call per step), timed after the headline
            "xrt_first_window": fw["xrt"] if fw else None,
            "first_window": fw,
            # the headline step with the temperature fallback on (5 temperatures x best_of
            # 5 re-decodes of every failing window, every window of the seek loop; rank 0's
            # figure, per GPU)
            "xrt_with_fallback": fb["xrt"] if fb else None,
            "fallback": fb,
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
                # the side that sets the overlapped step: the greedy decoder against its
                # HBM roofline (algorithmic bytes per position / decoder-side time per
                # position; launches per position from the captured decode graphs)
                "decoder": decoder_roofline(
                    pipe.whisper.cfg, dec_rows,
                    (calls if args.stagger else 1) * dec_positions,
                    (calls if args.stagger else 1) * dec_launches,
                    float(np.mean([b for _, b in sides])) if sides else None,
                    round(1.0 - cu_share, 4) if args.overlap > 0 else 1.0,
                    tkv_positions=(sets * dec_positions - 1) if args.stagger else None),
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args.model, float(np.mean(tok_counts)),
                                                   windows=float(np.mean(windows)) if windows else 1.0)
            except Exception as e:  # reported, never fatal to the bench line
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
