"""Batched Janus encode/decode on one GPU (the hot path of SURVEY.md §8, rows a1-a14).

Encode mirrors the engine glue ``process_audio_blocking`` / ``transmit_packet_blocking``
(backend/services/engine.py:510-552): per utterance transcribe (Whisper on the 48 kHz
buffer's ``[::3]``), prosody (YIN + RMS at 48 kHz, fallback Normal/Normal on error), and
— only if the text is non-empty (engine.py:536) — a ``JanusPacket(text, mode, prosody,
override_emotion=control_state.emotion_override)`` serialised to MessagePack bytes. The
engine's override is the str-enum ``"auto"``, so its packets carry ``'o': 'auto'``.

Decode mirrors the receiver (engine.py:220-280 -> Synthesizer.synthesize): deserialize,
build the "(emotion) text" prompt (synthesizer.py:149-177), then the GPU front end and
Firefly-GAN vocoder produce f32 audio and int16 PCM for all packets in one batch.
Morse packets stay on the host (synthesizer.py:257-326).
"""
import dataclasses
import os
import sys
import time
from typing import Optional

import numpy as np
import torch

from . import _native as nat
from .common.protocol import JanusMode, JanusPacket
from .services.prosody import ProsodyResult, prosody_launch
from .services.synthesizer import emotion_prompt
from .services.transcriber import TEMPERATURES
from .vocoder import DEFAULT_REFERENCE_ID, FireflyConfig, VocoderEngine, emotion_id
from .whisper import CONFIGS, WhisperEngine

CAPTURE_RATE = 48000


@dataclasses.dataclass
class ServingTuning:
    """Launch geometry of the serving steps; the defaults are the measured ones (DESIGN.md
    §5f-§5g, profiles/r04_* and r05_* A/Bs). The pipeline reads no environment: bench.py and
    the A/B tools build one with ``from_env`` (JANUS_<FIELD> in upper case) and pass it in."""
    persistent: int = 2             # staggered decoder: janus_decode_options.persistent
    stagger_sets: int = 2           # decoder slot sets per staggered call (>= 2)
    voc_dec_utts: int = 6           # staggered: packets rendered on the decoder's CUs
    yin_dec_utts: Optional[int] = None  # YIN utterances on the decoder side (None: the
                                    # staggered step's controller; 0 in the other steps)
    yin_beside: int = 128           # staggered: YIN grid cap beside the decoder (0 = after it)
    yin_side: str = "voc"           # overlapped step: "voc" (after the vocoder) or "beside"
    yin_blocks: int = 0             # overlapped step: YIN grid cap on the vocoder side (0 = none)
    yin_beside_blocks: int = 128    # overlapped step, yin_side "beside": its grid cap
    xattn_splits: Optional[int] = None  # cross-attention key splits (None: 1 staggered, 4 else)
    fallback_full: bool = True      # overlapped step: fallback re-decodes on the whole GPU
    fallback_xattn_splits: int = 4
    host_prefetch: bool = True      # staggered: D2H of the finished part behind the decoder
    side_timing: bool = False       # overlapped step: record per-side HIP events

    @classmethod
    def from_env(cls, env=None):
        """A tuning with every field JANUS_<NAME> sets in ``env`` (os.environ) overridden
        (tools and bench.py A/Bs only)."""
        env = os.environ if env is None else env
        kw = {}
        for f in dataclasses.fields(cls):
            v = env.get("JANUS_" + f.name.upper())
            if v is None:
                continue
            if f.name == "yin_side":
                kw[f.name] = v
            elif f.name in ("fallback_full", "host_prefetch", "side_timing"):
                kw[f.name] = v not in ("", "0")
            else:
                kw[f.name] = int(v)
        return cls(**kw)


class EncodeResult:
    """texts, tags, packets (bytes | None) per utterance, the decoded tokens, and
    ``stats``: f32 [B][3] device tensor (rms, mean voiced f0, voiced hops; NaN rows when
    prosody fell back, engine.py:520-525) for the result gather (dist.gather_results)."""

    def __init__(self, texts, tags, packets, tokens, n_tokens, stats=None, gates=None):
        self.texts, self.tags, self.packets = texts, tags, packets
        self.tokens, self.n_tokens = tokens, n_tokens
        self.stats = stats
        # per utterance: (needs_fallback at T = 0, no_speech_skip, avg_logprob, cr, nsp,
        # settled temperature, sampled fallback decodes)
        self.gates = gates


def _texts_and_gates(w, dec, temperatures=(0.0,), enc=None, **dec_kw):
    """Transcripts of one 30 s window per utterance plus faster-whisper's gates; a
    no-speech skip (no_speech_prob > 0.6 and avg_logprob <= -1) yields no text, as the
    reference's generate_segments skips the window (transcriber.py:53-64).
    ``temperatures`` beyond (0.0,): windows failing their gates go through
    generate_with_fallback (transcriber._fallback: sampled best_of-5 re-decodes of the
    encoder output ``enc``, on the caller's stream, ``dec_kw`` to decode_ex) and the
    settled result gives the text. Gates per utterance: (needs_fallback at T = 0,
    no_speech_skip, avg_logprob, compression_ratio, no_speech_prob, temperature, sampled
    decodes, seek after the window) of the settled result — the seek faster-whisper's
    generate_segments moves to (split_window: the window end, or the last timestamp pair);
    a seek short of the clip's content frames means the reference's loop decodes a second
    window from there (counted by bench.py as seek_windows_extra)."""
    from .services.transcriber import BEST_OF, N_FRAMES, _fallback, candidate, split_window
    tk = w.tokenizer
    first = [candidate(tk, toks, avg, nsp, 0.0) for (toks, avg, nsp) in dec.rows()]
    if len(temperatures) > 1:
        prompts = [list(tk.sot_sequence)] * len(first)
        final, ndec = _fallback(w, tk, enc, prompts, first, [(i, 0) for i in range(len(first))],
                                dec.tokens.shape[1], tuple(temperatures), BEST_OF, **dec_kw)
        texts = [tk.transcript(c.tokens) for c in final]
    else:
        final, ndec = first, [0] * len(first)
        texts = w.texts(dec.tokens, dec.prompt_lens)
    out_t, out_g = [], []
    for t, c0, c, nd in zip(texts, first, final, ndec):
        skip = c.no_speech_prob > 0.6 and not c.avg_logprob > -1.0
        out_t.append("" if skip else t)
        seek = N_FRAMES if skip else split_window(tk, c.tokens, 0, N_FRAMES)[1]
        out_g.append((c0.needs_fallback, skip, c.avg_logprob, c.compression_ratio, c.no_speech_prob,
                      c.temperature, nd, seek))
    return out_t, out_g


def _prosody_stats(parts, B, device):
    try:
        if parts and all(p is not None for p in parts):
            return torch.cat([torch.stack([p.rms[:len(p.hop_off) - 1], p.mean_f0[:len(p.hop_off) - 1],
                                           p.n_voiced[:len(p.hop_off) - 1].float()], 1) for p in parts])
    except Exception:
        pass
    return torch.full((B, 3), float("nan"), dtype=torch.float32, device=device)


def stagger_plan(sets, pos, started, k, S, fresh):
    """One staggered decoder call's plan (JanusPipeline.step_staggered), host-only: the
    first position of every slot set and the set whose batch completes in this call.
    sets[j]: None or {"born": call index the batch entered}; pos[j]: where set j's rows
    stand after the previous calls; k: this call's index (fresh set k % N); fresh: a new
    batch enters. Returns ([offset per set], completing set or None). A set holding a
    batch continues at (k - born) S (at most where its rows stand: the early exit stops a
    call whose rows all finished); a set without one continues from where its rows stand,
    at most (N-1) S, so it reads only tokens and KV rows it wrote; before the first call
    every set starts fresh. pos comes from the context (janus_whisper_decode_stand), which
    rejects any offset past it."""
    n = len(sets)
    f = k % n
    offs = [0] * n
    if started:
        for j in range(n):
            if j == f and fresh:
                offs[j] = 0
            elif sets[j] is not None:
                # (k - born) S, or less where every row finished early and the previous
                # call stopped short (its rows stand at pos[j]; the context rejects more)
                offs[j] = min((k - sets[j]["born"]) * S, pos[j])
            else:
                offs[j] = min(pos[j], (n - 1) * S)
    jc = (k - (n - 1)) % n
    done = jc if (sets[jc] is not None and k - sets[jc]["born"] == n - 1) else None
    return offs, done


class JanusPipeline:
    def __init__(self, model: str = "base.en", whisper_seed: int = 0, vocoder_seed: int = 0,
                 max_length: int = 448, vocoder_cfg: FireflyConfig = FireflyConfig(),
                 temperatures=TEMPERATURES, tuning: Optional[ServingTuning] = None):
        """temperatures: faster-whisper's fallback schedule (the default, as the
        reference's transcribe_buffer runs it); (0.0,) decodes each window once at T = 0
        and only reports the gates (bench.py's headline setting on synthetic weights,
        whose windows all fail the gates: DESIGN.md §0)."""
        self.device = nat.require_gpu()
        self.whisper = WhisperEngine(CONFIGS[model], seed=whisper_seed)
        self.vocoder = VocoderEngine(vocoder_cfg, seed=vocoder_seed)
        self._vocoder_seed = vocoder_seed
        self.max_length = max_length
        self.temperatures = tuple(float(t) for t in temperatures)
        # parity tests set this to read the encoder output back (it would otherwise keep
        # ~98 MB alive between calls at base.en, batch 64)
        self.keep_encoder_output = False
        self.last_encoder_output = None
        # serving-step geometry. The staggered step's decoder runs persistent segments
        # (janus_decode_options.persistent; 2 = one launch per layer step, 16 launches per
        # position: 246.5-248.5 vs 248.9-250.1 ms per step in three same-box rounds,
        # profiles/r05_layer_kernel_ab.txt)
        self.tuning = tuning if tuning is not None else ServingTuning()

    # ------------------------------------------------------------------ encode
    def encode(self, pcm: torch.Tensor, offsets: torch.Tensor, lengths, mode=JanusMode.SEMANTIC_VOICE,
               override="auto", timestamp=None) -> EncodeResult:
        B = len(lengths)
        w = self.whisper
        # prosody (YIN + RMS) does not depend on the transcript: it is enqueued first on
        # the caller's stream and runs beside the Whisper chain, which goes to a
        # high-priority stream — the greedy decoder is latency-bound and leaves most CUs
        # idle for YIN to fill (the decoder's early-exit checks block the host, so the
        # YIN launch must precede it)
        main = torch.cuda.current_stream(pcm.device)
        hi = self._hi_stream(pcm.device)
        hi.wait_stream(main)
        with torch.cuda.stream(hi):
            mel = w.logmel(pcm, offsets, B, 3)
            enc = w.encode(mel)
        if self.keep_encoder_output:   # [B][1500][d] fp16, for parity checks only
            self.last_encoder_output = enc
        main.wait_stream(hi)  # YIN after the (compute-bound) encoder, beside the decoder
        try:
            pres = prosody_launch(pcm, offsets, lengths, CAPTURE_RATE, 512, max_blocks=256)
        except Exception:  # engine.py:520-525
            pres = None
        with torch.cuda.stream(hi):
            dec = w.decode_ex(enc, max_length=self.max_length)
            texts, gts = _texts_and_gates(w, dec, self.temperatures, enc)
        main.wait_stream(hi)
        try:
            parts = pres if isinstance(pres, tuple) else (pres,)
            tags = None if any(p is None for p in parts) else [t for p in parts for t in p.tags()]
        except Exception:
            tags = None
        if tags is None:
            tags = [{"energy": "Normal", "pitch": "Normal"} for _ in range(B)]
        ts = time.time() if timestamp is None else timestamp
        packets = [JanusPacket(t, mode, g, override, ts).serialize() if t.strip() else None
                   for t, g in zip(texts, tags)]
        stats = _prosody_stats(parts if pres is not None else None, B, pcm.device)
        return EncodeResult(texts, tags, packets, dec.tokens, dec.n_tokens, stats, gts)

    def _xsplits(self, default):
        x = self.tuning.xattn_splits
        return default if x is None else x

    def _hi_stream(self, device):
        if getattr(self, "_hi", None) is None:
            self._hi = torch.cuda.Stream(device=device, priority=-1)
        return self._hi

    # ------------------------------------------------------------------ decode
    def set_reference_audio(self, wav: bytes = None):
        """The receiver's voice-cloning recording (synthesizer.py:67-104), or None. With a
        recording every packet is rendered in its voice (references=[...], :183-187,
        :243-247); without one SEMANTIC packets use the stock voice id (:189) and
        TEXT_ONLY packets none (references=None, :249)."""
        from .common.wavio import read_wav_16k
        self._ref_voice = (self.vocoder.speaker_embedding([read_wav_16k(wav)])[0]
                           if wav else None)

    def _voices(self, modes):
        v = self.vocoder
        if getattr(self, "_ref_voice", None) is not None:
            return self._ref_voice.expand(len(modes), -1)
        if getattr(self, "_stock_voice", None) is None:
            self._stock_voice = v.voice(DEFAULT_REFERENCE_ID)
        zero = torch.zeros_like(self._stock_voice)
        return torch.stack([self._stock_voice if m == JanusMode.SEMANTIC_VOICE else zero
                            for m in modes])

    def decode(self, packets, frames: int, vocoder=None):
        """packets: MessagePack bytes (None entries skipped). Returns (wav, pcm, prompts)
        for the SEMANTIC / TEXT_ONLY packets, all rendered to `frames` latent frames, in
        the voice the Synthesizer would request (set_reference_audio). ``vocoder``: another
        VocoderEngine with the same weights (its own workspaces: a second batch renders
        concurrently on another stream)."""
        voc = vocoder if vocoder is not None else self.vocoder
        prompts, emos, modes = [], [], []
        for p in packets:
            if p is None:
                continue
            pkt = JanusPacket.deserialize(p)
            if pkt.mode == JanusMode.MORSE_CODE:
                continue
            if pkt.mode == JanusMode.TEXT_ONLY:
                emo = pkt.override_emotion
                prompt, tag = ((f"({emo}) {pkt.text}", f"{emo}") if emo and emo != "Auto"
                               else (pkt.text, "relaxed"))
            else:
                prompt, tag = emotion_prompt(pkt)
            prompts.append(prompt.encode("utf-8"))
            emos.append(emotion_id(tag, self.vocoder.cfg.n_emotions))
            modes.append(pkt.mode)
        if not prompts:
            return None, None, []
        lat = voc.frontend(prompts, emos, frames, self._voices(modes))
        wav, pcm = voc.forward(lat)
        return wav, pcm, prompts

    def _vocoder_dec(self):
        """The second vocoder context (same seeded weights, own workspaces) that renders the
        decoder side's share of a staggered step's batch."""
        if getattr(self, "_voc2", None) is None:
            self._voc2 = VocoderEngine(self.vocoder.cfg, seed=self._vocoder_seed)
        return self._voc2

    def step(self, pcm, offsets, lengths, frames):
        enc = self.encode(pcm, offsets, lengths)
        wav, pcm16, _ = self.decode(enc.packets, frames)
        return enc, wav, pcm16

    # ------------------------------------------------------- overlapped (serving) step
    def _split_streams(self, device, dec_per_xcd: int):
        key = (str(device), dec_per_xcd)
        if getattr(self, "_split_key", None) != key:
            n = torch.cuda.get_device_properties(device).multi_processor_count
            dmask, vmask = nat.split_cu_masks(n, dec_per_xcd)
            self._dec_s = nat.MaskedStream(dmask, device)
            self._voc_s = nat.MaskedStream(vmask, device)
            # a second stream on the decoder's CUs: YIN beside the latency-bound decoder
            self._yin_s = nat.MaskedStream(dmask, device)
            self._split_key = key
            self._lane_key = None
        return self._dec_s.stream, self._voc_s.stream

    def step_overlapped(self, pcm, offsets, lengths, frames, dec_per_xcd: int = 16,
                        mode=JanusMode.SEMANTIC_VOICE, override="auto", timestamp=None):
        """One serving step of a two-stage pipeline: batch i goes through mel, encoder,
        greedy decoder and YIN; batch i-1 (kept from the previous call) through
        detokenisation, packets and the vocoder. Returns (EncodeResult, wav, pcm16) of
        batch i-1 — (None, None, None) on the first call; `flush` returns the last batch.

        Mel + encoder (compute-bound) get the whole GPU, and the host finishes batch i-1
        (transcripts, tags, MessagePack packets: a few ms) while they run. Then the greedy
        decoder of batch i (latency-bound) runs on a CU-masked stream holding
        `dec_per_xcd` CUs of each XCD, and the vocoder of batch i-1 followed by batch i's
        YIN on the disjoint rest, so neither holds the CUs the other needs (an unmasked
        overlap measured slower: the vocoder's long-running blocks delay every decoder
        launch)."""
        B = len(lengths)
        w = self.whisper
        main = torch.cuda.current_stream(pcm.device)
        hi = self._hi_stream(pcm.device)
        ds, vs = self._split_streams(pcm.device, dec_per_xcd)
        timing = self.tuning.side_timing
        # side_events (a list, set by the caller): each step appends its (vocoder side,
        # decoder side) HIP event pairs, recorded on the side streams without a host sync
        record = timing or getattr(self, "side_events", None) is not None
        yin_side = self.tuning.yin_side
        # YIN follows the vocoder on its own CUs: an uncapped grid lets the hardware balance
        # the uneven per-hop cost (early exit, silent hops) over them
        yin_blocks = self.tuning.yin_blocks

        def yin(u0=0, u1=B):
            try:
                return prosody_launch(pcm, offsets[u0:u1 + 1], lengths[u0:u1], CAPTURE_RATE, 512,
                                      max_blocks=yin_blocks)
            except Exception:  # engine.py:520-525
                return None
        # the YIN of the first tuning.yin_dec_utts utterances can run on the decoder side,
        # after the decoder, to even out the two sides (64 utterances, r02 v38: 2 / 6 / 8 /
        # 10 -> 316.7-317.1 / 314.5-315.2 / 313.6-314.3 / 315.2-315.7 ms per step; v40 with
        # the faster decoder: 8 / 12 / 16 -> 302.9-303.4 / 301.5-301.8 / 303.0-304.0; v42
        # with the fused merge + value projection (decoder side -3.4 ms) 16: the vocoder side
        # runs 286-301 ms from box to box, the decoder side 284-295; v46 with the C = 256
        # units on the register ring (vocoder side -7 ms): 16 / 10 / 6 -> 300.8-301.0 /
        # 298.4-298.9 / 297.4-298.9 ms on one box; 8; v49 with the faster encoder phase and
        # packed-pair YIN (1.14x): 8 / 4 / 0 -> 299.7-300.3 / 298.6-300.1 / 296.7-297.3 ms,
        # sides 284.7 / 282.0 ms at 0: all of YIN after the vocoder)
        n_dec = (min(B - 1, self.tuning.yin_dec_utts or 0)
                 if yin_side == "voc" else 0)
        ys = self._yin_s.stream if yin_side == "beside" else None
        pres = None
        hi.wait_stream(main)
        if yin_side == "early":  # on the vocoder's CUs, beside the (high-priority) encoder
            vs.wait_stream(main)
            with torch.cuda.stream(vs):
                pres = yin()
        with torch.cuda.stream(hi):
            mel = w.logmel(pcm, offsets, B, 3)
            enc = w.encode(mel)
        if self.keep_encoder_output:   # [B][1500][d] fp16 of batch i, for parity checks only
            self.last_encoder_output = enc
        # batch i-1 on the host while the encoder runs (its tensors were joined into the
        # caller's stream at the end of the previous call)
        prev = getattr(self, "_pending", None)
        self._pending = None
        res_prev = self._finish(*prev) if prev is not None else None
        # (the vocoder side starting beside the encoder instead: level, 248.9-249.3 vs
        # 248.6-248.9 ms, profiles/r05_host_prefetch_ab.txt)
        vs.wait_stream(hi)
        ds.wait_stream(hi)
        wav = pcm16 = None
        if record:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record(vs)
            ev[2].record(ds)
        with torch.cuda.stream(vs):
            if res_prev is not None:
                wav, pcm16, _ = self.decode(res_prev.packets, frames)
            if yin_side == "voc":
                pres = yin(n_dec, B)
            if record:
                ev[1].record(vs)  # before the decoder call, which blocks the host
        if ys is not None:  # YIN concurrently with the decoder, on its CUs, capped grid
            ys.wait_stream(hi)
            yin_cap = self.tuning.yin_beside_blocks
            with torch.cuda.stream(ys):
                try:
                    pres = prosody_launch(pcm, offsets, lengths, CAPTURE_RATE, 512, max_blocks=yin_cap)
                except Exception:  # engine.py:520-525
                    pres = None
        with torch.cuda.stream(ds):
            if yin_side == "dec":
                pres = yin()
            # 4 key splits per utterance on half the CUs (sweep 4/6/8/12/16: 313/315/327/330/339
            # ms); cu_count: the vocabulary projection at one block per CU of the partition
            # (128 vs 256 blocks: decoder side 308.6 -> 304.6 ms) and row-split skinny
            # projections from N <= 1024 (vs 2048: 310.5 -> 306.3 ms)
            dec_kw = dict(xattn_splits=self._xsplits(4),
                          cu_count=self._dec_s.n_cus)
            dec = w.decode_ex(enc, max_length=self.max_length, **dec_kw)
            # the fallback's sampled re-decodes (host-driven: reads the T = 0 gates); the
            # settled texts go to _finish. They run on the WHOLE GPU (the high-priority
            # stream, after the vocoder side and the T = 0 decode): the vocoder side ends
            # with the T = 0 decode anyway, and the 320-row cross-attention streams scale
            # with the CUs (tuning.fallback_full False: on the decoder's CUs, as the T = 0 decode)
            dec.settled = None
            if len(self.temperatures) > 1:
                if self.tuning.fallback_full:
                    hi.wait_stream(ds)
                    hi.wait_stream(vs)
                    fb_kw = dict(xattn_splits=self.tuning.fallback_xattn_splits,
                                 cu_count=torch.cuda.get_device_properties(pcm.device).multi_processor_count)
                    with torch.cuda.stream(hi):
                        dec.settled = _texts_and_gates(w, dec, self.temperatures, enc, **fb_kw)
                    ds.wait_stream(hi)
                else:
                    dec.settled = _texts_and_gates(w, dec, self.temperatures, enc, **dec_kw)
            if n_dec > 0:
                pres = (yin(0, n_dec), pres)
        if record:
            ev[3].record(ds)
            if getattr(self, "side_events", None) is not None:
                self.side_events.append(ev)
        main.wait_stream(ds)
        main.wait_stream(vs)
        if ys is not None:
            main.wait_stream(ys)
        if timing:
            torch.cuda.synchronize()
            print(f"[overlap] vocoder side {ev[0].elapsed_time(ev[1]):.1f} ms, decoder side "
                  f"{ev[2].elapsed_time(ev[3]):.1f} ms", file=sys.stderr, flush=True)
        self._pending = (dec, pres, B, mode, override, timestamp)
        return res_prev, wav, pcm16

    def _finish(self, dec, pres, B, mode, override, timestamp) -> EncodeResult:
        """Host tail of an encode: transcripts, prosody tags (fallback Normal/Normal,
        engine.py:520-525), packets (engine.py:527-548)."""
        host = getattr(dec, "host", None)
        if host is not None:   # copies issued behind the decoder call (_host_prefetch)
            ev, hdec, hpres = host
            ev.synchronize()
        try:
            parts = pres if isinstance(pres, tuple) else (pres,)
            if host is not None and hpres is not None:
                tags = [t for (r, m, v) in hpres for t in ProsodyResult.tags_of(r.numpy(), m.numpy(), v.numpy())]
            else:
                tags = None if any(p is None for p in parts) else [t for p in parts for t in p.tags()]
        except Exception:
            tags = None
        if tags is None:
            tags = [{"energy": "Normal", "pitch": "Normal"} for _ in range(B)]
        settled = getattr(dec, "settled", None)
        texts, gts = settled if settled is not None else _texts_and_gates(
            self.whisper, hdec if host is not None else dec)
        ts = time.time() if timestamp is None else timestamp
        packets = [JanusPacket(t, mode, g, override, ts).serialize() if t.strip() else None
                   for t, g in zip(texts, tags)]
        stats = _prosody_stats(parts if pres is not None else None, B, dec.tokens.device)
        return EncodeResult(texts, tags, packets, dec.tokens, dec.n_tokens, stats, gts)

    def _host_prefetch(self, part, pres, st, stream):
        """Device-to-host copies of what _finish reads of a completing batch (its tokens,
        counts, log-probs, no-speech probabilities and YIN statistics), issued on `stream`
        right behind the decoder call that completed it, into pinned buffers. _finish then
        waits for that call alone — not, through the caller's stream, for the vocoder side
        that ends later — so the host tail (detokenising, gates, packets) overlaps the
        vocoder's last milliseconds. One buffer set: the next call's copies are enqueued
        after this host tail has read them. The copies run on a torch-owned stream behind
        `stream` (the pinned blocks' lifetime events then never sit on a CU-masked stream
        that is destroyed before them at exit)."""
        from .whisper import DecodeOut
        hb = st.setdefault("hbuf", {})
        cs = getattr(self, "_d2h_stream", None)
        if cs is None:
            cs = self._d2h_stream = torch.cuda.Stream(part.tokens.device)
        cs.wait_stream(stream)
        stream = cs

        def pin(name, t):
            buf = hb.get(name)
            if buf is None or buf.shape != t.shape or buf.dtype != t.dtype:
                buf = hb[name] = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            buf.copy_(t, non_blocking=True)
            return buf
        with torch.cuda.stream(stream):
            hdec = DecodeOut(pin("tok", part.tokens), pin("nt", part.n_tokens), pin("lp", part.sum_logprob),
                             pin("ns", part.no_speech_prob), part.prompt_lens)
            parts = pres if isinstance(pres, tuple) else (pres,)
            hpres = None
            if all(p is not None for p in parts):
                hpres = [(pin(f"rms{i}", p.rms), pin(f"mf{i}", p.mean_f0), pin(f"nv{i}", p.n_voiced))
                         for i, p in enumerate(parts)]
            ev = torch.cuda.Event()
            ev.record(stream)
        return ev, hdec, hpres

    # ------------------------------------------- staggered (continuous-batching) step
    def step_staggered(self, pcm, offsets, lengths, frames, dec_per_xcd: int = 16,
                       mode=JanusMode.SEMANTIC_VOICE, override="auto", timestamp=None):
        """The overlapped serving step with the greedy decoder as a continuous batch of N
        batches at different positions (janus_decode_rows.pos_offset; N =
        tuning.stagger_sets, default 2): each call of the decoder advances N·B rows by
        S = max_length // N positions — batch i's rows fresh (positions 0 .. S-1) and
        batch i-m's, m = 1 .. N-1, continuing in their slot set (positions mS .. (m+1)S-1),
        so every step still completes exactly one batch's decode, but the decoder's
        latency-bound launches serve N times the rows. Per step: mel + encoder of batch i
        (whole GPU), then the decoder call on the decoder's CUs (with the YIN of the first
        n_dec utterances of batch i beside it, _yin_split) beside the vocoder of batch i-N
        + the rest of batch i's YIN on the vocoder's CUs. Returns (EncodeResult, wav, pcm16) of
        batch i-N, (None, None, None) for the first N calls; ``flush_staggered`` drains.
        The continuous batch decodes at T = 0; per-row results are bit-identical to the
        one-batch decode (rows are independent of their neighbours' positions). With the
        temperature fallback on (``temperatures`` beyond (0.0,), faster-whisper's default),
        the windows of the completing batch that fail their gates leave the continuous
        batch: their sampled best_of re-decodes (generate_with_fallback) run at the end of
        the call on the whole GPU, from the batch's encoder output still in its slot set,
        in decoder state slot 1 (the continuous batch's slots stay untouched in slot 0), as
        step_overlapped runs them."""
        B = len(lengths)
        w = self.whisper
        L = self.max_length
        dev = pcm.device if pcm is not None else self.device
        main = torch.cuda.current_stream(dev)
        hi = self._hi_stream(dev)
        ds, vs = self._split_streams(dev, dec_per_xcd)
        st = getattr(self, "_stag", None)
        if st is not None and st["B"] != B:
            # the slot layout (and every KV / token row in it) is sized by B: batches still
            # in the decoder would be lost
            if any(x is not None for x in st["sets"]) or st["done"] is not None:
                raise ValueError(f"step_staggered: batch size {B} != {st['B']} while batches are "
                                 "in flight; call flush_staggered() first (or pad the batch)")
            st = None
        if st is None:
            n = max(2, self.tuning.stagger_sets)
            d = w.cfg.d_model
            st = self._stag = {"B": B, "n": n, "k": 0, "sets": [None] * n, "done": None,
                               "enc": torch.zeros(n * B, w.cfg.n_audio_ctx, d, dtype=torch.float16,
                                                  device=dev)}
        n, k = st["n"], st["k"]
        # S positions per call cover the full decode's L - 1 steps in N calls; the last set's
        # chunk may overrun by a position (a no-op past the row's end) but not past L
        S = -(-(L - 1) // n)
        if n * S > L:
            raise ValueError(f"stagger_sets={n} does not tile max_length {L}")
        f = k % n   # this call's fresh slot set (its last batch completed in the previous call)
        hi.wait_stream(main)
        with torch.cuda.stream(hi):
            if pcm is not None:
                mel = w.logmel(pcm, offsets, B, 3)
                st["enc"][f * B:(f + 1) * B].copy_(w.encode(mel))
        # batch i-N (completed by the previous call) on the host while the encoder runs
        prev = st["done"]
        st["done"] = None
        res_prev = self._finish(*prev) if prev is not None else None
        vs.wait_stream(hi)
        ds.wait_stream(hi)
        record = getattr(self, "side_events", None) is not None
        # side events every step: the YIN split below reads the previous step's
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record(vs)
        ev[2].record(ds)
        wav = pcm16 = None
        pres = None
        # YIN of the first n_dec utterances runs on the decoder side (beside the decoder call,
        # below), the rest behind the vocoder: with two batches per decoder call that side has
        # the slack (64 x 30 s, one box, YIN after the call: 0 / 24 / 32 / 40 of 64 -> sides
        # 275 / 242, 260 / 246, 256 / 249, 253 / 253 ms; step 287 -> 264 ms)
        n_dec = self._yin_split(st, B) if pcm is not None else 0

        def yin(u0, u1):
            try:
                return prosody_launch(pcm, offsets[u0:u1 + 1], lengths[u0:u1], CAPTURE_RATE, 512,
                                      max_blocks=0)
            except Exception:  # engine.py:520-525
                return None
        # the last kv packets of the batch render on the decoder's CUs after its call (a
        # second vocoder context), the rest here: a decoder side that finishes early takes
        # vocoder work the way the vocoder side takes YIN (tuning.voc_dec_utts; with the r05
        # decoder segments: 3 / 4 / 5 -> 252.2-252.7 / 251.2-251.3 / 251.9-252.3 ms per step,
        # profiles/r05_voc_dec_sweep2.txt; with the layer-step grid and the DPP reductions the
        # decoder side has slack at 4 (YIN split pinned at 63): 4 / 5 / 6 / 8 -> 246.4-247.7 /
        # 244.7-245.4 / 245.7-246.8 / 249.3-249.8, profiles/r05_voc_dec_sweep3.txt; with the
        # decoder's waves at priority 3 over the YIN blocks beside them, 6: see mfma.h
        # JANUS_DEC_PRIO)
        kv = 0
        pk_dec = []
        wav_b = pcm_b = None
        with torch.cuda.stream(vs):
            if res_prev is not None:
                pk = res_prev.packets
                kv = min(len(pk), max(0, self.tuning.voc_dec_utts))
                self.voc_dec_utts = kv   # the main vocoder context renders the other len(pk) - kv
                pk_dec = pk[len(pk) - kv:] if kv else []
                wav, pcm16, _ = self.decode(pk[:len(pk) - kv], frames)
            if pcm is not None:
                pres = yin(n_dec, B)
            ev[1].record(vs)
        # each set's first position: the fresh set 0, a set holding the batch that entered at
        # call b (k - b) S; the first call starts every set fresh (no set holds state yet);
        # later a set without a batch runs as continuing rows over the state it holds, from
        # where its rows stand (at most (N-1) S: a finished set re-runs its last chunk), so
        # every token and KV-cache row it reads was written (its output is not read)
        pos = st.setdefault("pos", [0] * n)
        set_offs, jc = stagger_plan(st["sets"], pos, bool(st.get("started")), k, S, pcm is not None)
        offs = [o for o in set_offs for _ in range(B)]
        cont = st["sets"][jc] if jc is not None else None
        dec = None
        host = None
        if pcm is not None or any(x is not None for x in st["sets"]):
            with torch.cuda.stream(ds):
                # cross-attention at ONE key split (r05): with 2 x 64 rows the grid fills the
                # decoder's CUs without splitting the keys, and at one split the kernel writes
                # its output itself (no merge launch: 81 -> 75 launches per position; decoder
                # side 246.2 / 244.4 -> 243.8 / 242.0 ms in two same-box rounds,
                # profiles/r05_xattn_split1_ab.txt; r04: 4 splits 252.6-255.3, 2 246.7-248.6,
                # 8 264.7-266.7 ms)
                # the decoder side's YIN runs concurrently with the decode call, on a second
                # stream over the decoder's CUs with its grid capped at tuning.yin_beside
                # blocks (default 128; 0: after the call): the latency-bound decoder leaves
                # issue slots free. Same box, two rounds of 5 steps: 259.4 / 258.4 ms at 128
                # against 261.7 / 262.3 after the call and 263.0 / 262.3 at 256
                # (profiles/r04_yin_beside_ab.json)
                yb = self.tuning.yin_beside
                beside = yb > 0 and n_dec > 0
                if beside:
                    ys = self._yin_s.stream
                    ys.wait_stream(ds)
                    with torch.cuda.stream(ys):
                        try:
                            pd = prosody_launch(pcm, offsets[0:n_dec + 1], lengths[0:n_dec], CAPTURE_RATE,
                                                512, max_blocks=yb)
                        except Exception:  # engine.py:520-525
                            pd = None
                dec = w.decode_ex(st["enc"], max_length=L, pos_offset=offs, steps=S,
                                  xattn_splits=self._xsplits(1),
                                  cu_count=self._dec_s.n_cus, persistent=self.tuning.persistent)
                if cont is not None and len(self.temperatures) == 1 and self.tuning.host_prefetch:
                    from .whisper import DecodeOut
                    sl = slice(jc * B, (jc + 1) * B)
                    hpart = DecodeOut(dec.tokens[sl], dec.n_tokens[sl], dec.sum_logprob[sl],
                                      dec.no_speech_prob[sl], dec.prompt_lens[sl])
                    host = self._host_prefetch(hpart, cont["pres"], st, ds)
                if beside:
                    ds.wait_stream(ys)
                    pres = (pd, pres)
                elif n_dec > 0:
                    pres = (yin(0, n_dec), pres)
            st["started"] = True
            # where each set's rows stand now (offset + S, or fewer when every row
            # finished and the call stopped early), as the context recorded it
            stand = w.decode_stand(n * B)
            for j in range(n):
                pos[j] = stand[j * B]
        if pk_dec:
            with torch.cuda.stream(ds):
                wav_b, pcm_b, _ = self.decode(pk_dec, frames, vocoder=self._vocoder_dec())
        if pcm is not None:
            st["sets"][f] = {"pres": pres, "B": B, "mode": mode, "override": override,
                             "timestamp": timestamp, "born": k}
        ev[3].record(ds)
        if record:
            self.side_events.append(ev)
        # only full steps (a vocoder batch, a batch completing) steer the YIN split
        if pcm is not None and res_prev is not None and cont is not None:
            st["prev_ev"] = ev
        main.wait_stream(ds)
        main.wait_stream(vs)
        if wav_b is not None:   # the batch back in packet order
            wav = wav_b if wav is None else torch.cat([wav, wav_b])
            pcm16 = pcm_b if pcm16 is None else torch.cat([pcm16, pcm_b])
        if cont is not None:
            sl = slice(jc * B, (jc + 1) * B)
            from .whisper import DecodeOut
            part = DecodeOut(dec.tokens[sl], dec.n_tokens[sl], dec.sum_logprob[sl],
                             dec.no_speech_prob[sl], dec.prompt_lens[sl])
            part.settled = None
            if host is not None:
                part.host = host
            if len(self.temperatures) > 1:
                # the fallback of the completing batch's failing windows, on the whole GPU
                # after both sides (its encoder output stays in slot set jc until the next
                # call's encoder, later on the same stream, overwrites it)
                hi.wait_stream(main)
                fb_kw = dict(xattn_splits=self.tuning.fallback_xattn_splits,
                             cu_count=torch.cuda.get_device_properties(dev).multi_processor_count,
                             state_slot=1)
                with torch.cuda.stream(hi):
                    part.settled = _texts_and_gates(w, part, self.temperatures, st["enc"][sl], **fb_kw)
                main.wait_stream(hi)
            st["done"] = (part, cont["pres"], B, cont["mode"], cont["override"], cont["timestamp"])
            st["sets"][jc] = None
        st["k"] = k + 1
        return res_prev, wav, pcm16

    # YIN of one 30 s utterance on a 16-CU-per-XCD partition (26 ms for 64, either side)
    YIN_MS_PER_UTT = 0.4

    def _yin_split(self, st, B):
        """Utterances whose YIN runs on the decoder side in the staggered step. Fixed by
        tuning.yin_dec_utts; otherwise self-balancing: starts at 7B/8 (where it settled on
        the r04 boxes: 52-59 of 64) and moves by the previous full step's side-time gap
        (vocoder side minus decoder side, HIP events on the two CU-masked streams) over
        twice the per-utterance YIN time, at most 16 per step,
        so the two partitions finish together whatever the box's vocoder / decoder speed
        ratio (measured from box to box: vocoder side 253-265 ms at the same split)."""
        if self.tuning.yin_dec_utts is not None:
            return max(0, min(B - 1, self.tuning.yin_dec_utts))
        n = st.get("n_dec", 7 * B // 8)
        prev = st.get("prev_ev")
        if prev is not None and prev[1].query() and prev[3].query():
            gap = prev[0].elapsed_time(prev[1]) - prev[2].elapsed_time(prev[3])
            move = int(round(gap / (2.0 * self.YIN_MS_PER_UTT)))
            n = max(0, min(B - 1, n + max(-16, min(16, move))))
        st["n_dec"] = n
        return n

    def flush_staggered(self, frames):
        """Drain the staggered pipeline: finish the batches still in the decoder and render
        them. Returns a list of (EncodeResult, wav, pcm16), in order."""
        out = []
        st = getattr(self, "_stag", None)
        if st is None:
            return out
        while any(x is not None for x in st["sets"]):
            r = self.step_staggered(None, None, [0] * st["B"], frames)
            if r[0] is not None:
                out.append(r)
        prev, st["done"] = st["done"], None
        if prev is not None:
            res = self._finish(*prev)
            wav, pcm16, _ = self.decode(res.packets, frames)
            out.append((res, wav, pcm16))
        self._stag = None
        return out

    # ------------------------------ three-lane step: the encoder off the critical path
    def _lane_streams(self, device, dec_per_xcd: int, enc_per_xcd: int):
        key = (str(device), dec_per_xcd, enc_per_xcd)
        if getattr(self, "_lane_key", None) != key:
            n = torch.cuda.get_device_properties(device).multi_processor_count
            if enc_per_xcd > 0:
                dmask, emask, vmask = nat.group_cu_masks(
                    n, [dec_per_xcd - enc_per_xcd, enc_per_xcd, n // 8 - dec_per_xcd])
            else:   # 0: the encoder shares the decoder's CUs on a stream of its own
                dmask, vmask = nat.split_cu_masks(n, dec_per_xcd)
                emask = dmask
            self._dec_s = nat.MaskedStream(dmask, device)
            self._enc_s = nat.MaskedStream(emask, device)
            self._voc_s = nat.MaskedStream(vmask, device)
            self._lane_key = key
            self._split_key = None
        return self._dec_s.stream, self._enc_s.stream, self._voc_s.stream

    def step_pipelined(self, pcm, offsets, lengths, frames, dec_per_xcd: int = 16,
                       enc_per_xcd: int = 4, mode=JanusMode.SEMANTIC_VOICE, override="auto",
                       timestamp=None):
        """The staggered serving step with the encoder moved OFF the critical path: three
        CU-disjoint lanes run side by side for the whole step —
          encoder lane (``enc_per_xcd`` CUs of each XCD, carved out of the decoder's
            ``dec_per_xcd``; 0: a stream of its own on the decoder's CUs, filling the
            latency-bound decoder's idle issue slots): mel + encoder of batch i into a
            staging buffer;
          decoder lane (the other dec_per_xcd - enc_per_xcd): ONE continuous-batch decode
            call of batch i-1 (fresh, positions 0 .. S-1, its encoder output copied out of
            the staging buffer first) and batch i-2 (continuing, positions S .. 2S-1);
          vocoder lane (the rest): the vocoder of batch i-3 (finished on the host at the
            end of the previous call), then YIN of batch i.
        The host finishes batch i-2 (transcripts, tags, packets) as soon as the decoder lane
        is done, inside the vocoder lane's time. Returns (EncodeResult, wav, pcm16) of batch
        i-3 ((None, None, None) for the first three calls); ``flush_pipelined`` drains.
        Greedy (T = 0) only; per-row results are those of the one-batch decode (the
        staggered decode's parity, and the encoder is the same kernels on fewer CUs)."""
        if tuple(self.temperatures) != (0.0,):
            raise NotImplementedError("pipelined step runs at temperature 0 only")
        B = len(lengths)
        w = self.whisper
        L = self.max_length
        S = L // 2
        dev = pcm.device if pcm is not None else self.device
        main = torch.cuda.current_stream(dev)
        ds, es, vs = self._lane_streams(dev, dec_per_xcd, enc_per_xcd)
        st = getattr(self, "_lanes", None)
        if st is not None and st["B"] != B:
            if (st["staged"] is not None or st["vocode"] is not None
                    or any(x is not None for x in st["sets"])):
                raise ValueError(f"step_pipelined: batch size {B} != {st['B']} while batches are "
                                 "in flight; call flush_pipelined() first (or pad the batch)")
            st = None
        if st is None:
            d = w.cfg.d_model
            st = self._lanes = {"B": B, "parity": 0, "sets": [None, None], "staged": None,
                                "vocode": None, "started": False, "pos": [0, 0],
                                "enc": torch.zeros(2 * B, w.cfg.n_audio_ctx, d, dtype=torch.float16,
                                                   device=dev),
                                "stage": torch.zeros(B, w.cfg.n_audio_ctx, d, dtype=torch.float16,
                                                     device=dev)}
        f = st["parity"]
        c = 1 - f
        for x in (ds, es, vs):
            x.wait_stream(main)
        record = getattr(self, "side_events", None) is not None
        if record:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
            ev[0].record(vs)
            ev[2].record(ds)
            ev[4].record(es)
        staged, cont = st["staged"], st["sets"][c]
        # enqueue order matters: the decoder call can hold the host until its lane has
        # drained what is queued ahead of it, so the vocoder and encoder lanes are filled
        # first (measured: the vocoder lane queued behind the decoder call ran serially)
        # decoder lane, first: batch i-1's encoder output out of the staging buffer into its
        # slot set (the encoder lane overwrites the stage only after this copy)
        copied = torch.cuda.Event()
        with torch.cuda.stream(ds):
            if staged is not None:
                st["enc"][f * B:(f + 1) * B].copy_(st["stage"])
            copied.record(ds)
        n_dec = min(B - 1, self.tuning.yin_dec_utts or 0) if pcm is not None else 0

        def yin(u0, u1):
            try:
                return prosody_launch(pcm, offsets[u0:u1 + 1], lengths[u0:u1], CAPTURE_RATE, 512,
                                      max_blocks=0)
            except Exception:  # engine.py:520-525
                return None
        # vocoder lane: the batch the host finished at the end of the previous call, then
        # YIN of batch i (all but the first n_dec utterances)
        res_prev = st["vocode"]
        st["vocode"] = None
        wav = pcm16 = None
        rest = None
        with torch.cuda.stream(vs):
            if res_prev is not None:
                wav, pcm16, _ = self.decode(res_prev.packets, frames)
            if pcm is not None:
                rest = yin(n_dec, B)
            if record:
                ev[1].record(vs)
        # encoder lane: batch i
        with torch.cuda.stream(es):
            es.wait_event(copied)
            if pcm is not None:
                mel = w.logmel(pcm, offsets, B, 3)
                st["stage"].copy_(w.encode(mel))
            if record:
                ev[5].record(es)
        # decoder lane: fresh rows (set f) start at 0, the continuing set at S; a set with no
        # batch runs as continuing rows over the finished state it holds (output unread)
        dec = None
        if staged is not None or cont is not None:
            started = st["started"]
            offs = [0] * (2 * B)
            for k in range(2 * B):
                if k // B == f:
                    offs[k] = 0 if staged is not None or not started else L - S
                else:
                    offs[k] = S if cont is not None else (L - S if started else 0)
                if offs[k] > 0:   # never past where the slot stands (early-exit calls)
                    offs[k] = min(offs[k], st["pos"][k // B])
            with torch.cuda.stream(ds):
                dec = w.decode_ex(st["enc"], max_length=L, pos_offset=offs, steps=S,
                                  xattn_splits=self._xsplits(4),
                                  cu_count=self._dec_s.n_cus)
            stand = w.decode_stand(2 * B)
            st["pos"] = [stand[0], stand[B]]
            st["started"] = True
        pres = rest
        with torch.cuda.stream(ds):
            if n_dec > 0:
                pres = (yin(0, n_dec), rest)
            if record:
                ev[3].record(ds)
        if record:
            self.side_events.append(ev)
        # host: batch i-2 is complete once the decoder lane is; finish it on the decoder
        # lane's stream (its copies then wait for that lane only) while the vocoder lane
        # runs (its YIN ran two calls ago)
        st["sets"][f] = staged
        if cont is not None:
            sl = slice(c * B, (c + 1) * B)
            from .whisper import DecodeOut
            part = DecodeOut(dec.tokens[sl], dec.n_tokens[sl], dec.sum_logprob[sl],
                             dec.no_speech_prob[sl], dec.prompt_lens[sl])
            with torch.cuda.stream(ds):
                st["vocode"] = self._finish(part, cont["pres"], B, cont["mode"], cont["override"],
                                            cont["timestamp"])
        st["sets"][c] = None
        st["parity"] = c
        st["staged"] = (None if pcm is None else {"pres": pres, "B": B, "mode": mode,
                                                  "override": override, "timestamp": timestamp})
        for x in (ds, es, vs):
            main.wait_stream(x)
        return res_prev, wav, pcm16

    def flush_pipelined(self, frames):
        """Drain the three-lane pipeline: list of (EncodeResult, wav, pcm16) for the batches
        still in it, in order."""
        out = []
        st = getattr(self, "_lanes", None)
        if st is None:
            return out
        while (st["staged"] is not None or st["vocode"] is not None
               or any(x is not None for x in st["sets"])):
            r = self.step_pipelined(None, None, [0] * st["B"], frames,
                                    *(self._lane_key[1:] if getattr(self, "_lane_key", None) else ()))
            if r[0] is not None:
                out.append(r)
        self._lanes = None
        return out

    def flush(self, frames):
        """Finish and render the batch the last overlapped step left pending:
        (EncodeResult, wav, pcm16), or (None, None, None)."""
        prev, self._pending = getattr(self, "_pending", None), None
        if prev is None:
            return None, None, None
        res = self._finish(*prev)
        wav, pcm16, _ = self.decode(res.packets, frames)
        return res, wav, pcm16
