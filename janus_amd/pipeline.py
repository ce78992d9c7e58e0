"""Batched Janus encode/decode on one GPU (the hot path of SURVEY.md §8, rows a1-a14).

Encode mirrors the engine glue ``process_audio_blocking`` / ``transmit_packet_blocking``
(backend/services/engine.py:510-552): per utterance transcribe (Whisper on the 48 kHz
buffer's ``[::3]``, faster-whisper's whole seek loop as ``transcribe_buffer`` runs it,
transcriber.py:29-64: every 30 s window from the seek the previous window ended at, each
window's segments joined), prosody (YIN + RMS at 48 kHz, fallback Normal/Normal on error),
and — only if the text is non-empty (engine.py:536) — a ``JanusPacket(text, mode, prosody,
override_emotion=control_state.emotion_override)`` serialised to MessagePack bytes. The
engine's override is the str-enum ``"auto"``, so its packets carry ``'o': 'auto'``.

Decode mirrors the receiver (engine.py:220-280 -> Synthesizer.synthesize): deserialize,
build the "(emotion) text" prompt (synthesizer.py:149-177), then the GPU front end and
Firefly-GAN vocoder produce f32 audio and int16 PCM for all packets in one batch.
Morse packets stay on the host (synthesizer.py:257-326).
"""
import collections
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
from .services.transcriber import (BEST_OF, HOP, N_FRAMES, TEMPERATURES, _Stream, advance,
                                   gather_windows, settle_round)
from .vocoder import DEFAULT_REFERENCE_ID, FireflyConfig, VocoderEngine, emotion_id
from .whisper import CONFIGS, WhisperEngine

CAPTURE_RATE = 48000


@dataclasses.dataclass
class ServingTuning:
    """Launch geometry of the serving steps; the defaults are the measured ones (DESIGN.md
    §5f-§5h, profiles/r04_* .. r06_* A/Bs). The pipeline reads no environment: bench.py and
    the A/B tools build one with ``from_env`` (JANUS_<FIELD> in upper case) and pass it in."""
    persistent: int = 2             # staggered decoder: janus_decode_options.persistent
    stagger_sets: int = 2           # decoder slot sets per staggered call (>= 2)
    all_windows: bool = True        # the whole seek loop (False: each clip's first window only,
                                    # the r05 serving semantics, kept as a comparison leg)
    set_batches: int = 0            # staggered: rows per decoder slot set, in batches of B
                                    # (0: 2 with all_windows — a batch's first windows and an
                                    # earlier batch's continuation windows enter together —, 1
                                    # without)
    calls_per_step: int = 0         # staggered decoder calls per step (0: the windows a step
                                    # takes in, 2 per clip with all_windows, / set_batches)
    cont_encode: str = "hi"         # staggered: continuation windows encoded on the whole GPU
                                    # before this step's call ("hi"), or on the vocoder's CUs,
                                    # entering the next step's call ("voc": its traffic beside
                                    # the decoder costs more, 344.9 vs 333.8 ms per step,
                                    # profiles/r06_cont_encode_ab.txt)
    voc_dec_utts: int = 0           # staggered: packets rendered on the decoder's CUs
    yin_dec_utts: Optional[int] = None  # YIN utterances on the decoder side (None: the
                                    # staggered step's controller; 0 in the other steps)
    yin_beside: int = 128           # staggered: YIN grid cap beside the decoder (0 = after it)
    yin_side: str = "voc"           # overlapped step: "voc" (after the vocoder) or "beside"
    yin_blocks: int = 0             # overlapped step: YIN grid cap on the vocoder side (0 = none)
    yin_beside_blocks: int = 128    # overlapped step, yin_side "beside": its grid cap
    xattn_splits: Optional[int] = None  # cross-attention key splits (None: 1 staggered, 4 else)
    dec_path_flags: int = 0         # staggered decoder: janus_decode_options.path_flags (A/Bs)
    dec_poll: int = 16              # staggered decoder: janus_decode_options.check_every (0: the
                                    # calls do not wait for their stream — measured 50 % slower,
                                    # DESIGN.md §5h)
    logits_blocks: int = 0          # staggered decoder: vocabulary-projection blocks per row
                                    # group of 64 (janus_decode_options.logits_blocks; 0: the
                                    # decoder's CUs / row groups, so every group runs in ONE
                                    # round and its blocks of a vocabulary slice share an L2:
                                    # 32 at 256 rows, +1.6 % xRT against one block per CU,
                                    # DESIGN.md §5h)
    fallback_full: bool = True      # overlapped step: seek rounds / fallback on the whole GPU
    fallback_xattn_splits: int = 4
    host_prefetch: bool = True      # staggered: D2H of the completed windows behind their call
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
            if f.name in ("yin_side", "cont_encode"):
                kw[f.name] = v
            elif f.name in ("fallback_full", "host_prefetch", "side_timing", "all_windows"):
                kw[f.name] = v not in ("", "0")
            else:
                kw[f.name] = int(v)
        return cls(**kw)

    def batches_per_set(self):
        return self.set_batches if self.set_batches > 0 else (2 if self.all_windows else 1)

    def calls(self):
        if self.calls_per_step > 0:
            return self.calls_per_step
        return max(1, (2 if self.all_windows else 1) // self.batches_per_set())


class EncodeResult:
    """texts, tags, packets (bytes | None) per utterance; ``streams``: each utterance's
    seek-loop state (segments, windows, counters, the settled tokens of every window);
    ``tokens`` / ``n_tokens``: the FIRST window's decode (int32 [B][max_length] with the
    prompt, sampled counts); ``sampled``: tokens sampled at T = 0 over every window; ``stats``:
    f32 [B][3] device tensor (rms, mean voiced f0, voiced hops; NaN rows when prosody fell
    back, engine.py:520-525) for the result gather (dist.gather_results); ``gates`` per
    utterance, of its first window: (needs_fallback at T = 0, no_speech_skip, avg_logprob,
    compression_ratio, no_speech_prob, settled temperature, sampled re-decodes, seek after
    the window)."""

    def __init__(self, texts, tags, packets, tokens, n_tokens, stats=None, gates=None, streams=None):
        self.texts, self.tags, self.packets = texts, tags, packets
        self.tokens, self.n_tokens = tokens, n_tokens
        self.stats = stats
        self.gates = gates
        self.streams = streams

    @property
    def windows(self):
        return [s.windows for s in self.streams] if self.streams is not None else None

    @property
    def sampled(self):
        return [s.sampled for s in self.streams] if self.streams is not None else None


def _prosody_stats(parts, B, device):
    try:
        if parts and all(p is not None for p in parts):
            return torch.cat([torch.stack([p.rms[:len(p.hop_off) - 1], p.mean_f0[:len(p.hop_off) - 1],
                                           p.n_voiced[:len(p.hop_off) - 1].float()], 1) for p in parts])
    except Exception:
        pass
    return torch.full((B, 3), float("nan"), dtype=torch.float32, device=device)


def _tags(pres, host, B):
    """Prosody tags of a batch (fallback Normal/Normal on any error, engine.py:520-525);
    ``host``: pinned copies of the stats (_prefetch_stats) or None."""
    try:
        parts = pres if isinstance(pres, tuple) else (pres,)
        if host is not None:
            ev, hp = host
            ev.synchronize()
            tags = [t for (r, m, v) in hp for t in ProsodyResult.tags_of(r.numpy(), m.numpy(), v.numpy())]
        else:
            tags = None if any(p is None for p in parts) else [t for p in parts for t in p.tags()]
    except Exception:
        tags = None
    return tags if tags is not None else [{"energy": "Normal", "pitch": "Normal"} for _ in range(B)]


def contents_of(lengths):
    """Content frames of each clip's 16 kHz view (len(x[::3]) // 160), as faster-whisper
    counts them for the 48 kHz buffer's [::3] (transcriber.py:51-57)."""
    return [((int(n) + 2) // 3) // HOP for n in lengths]


def stagger_plan(sets, pos, started, k, S, fresh):
    """One staggered decoder call's plan (JanusPipeline.step_staggered), host-only: the
    first position of every slot set and the set whose group completes in this call.
    sets[j]: None or {"born": call index the group entered}; pos[j]: where set j's rows
    stand after the previous calls; k: this call's index (fresh set k % N); fresh: a new
    group enters. Returns ([offset per set], completing set or None). A set holding a
    group continues at (k - born) S (at most where its rows stand: the early exit stops a
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


class _Batch:
    """One serving batch in flight: its clips' seek-loop states, whole-clip features (fp16
    [B][F][80] on the GPU, kept until the last window of the batch has entered the decoder)
    and prosody, until every clip's last window has settled."""

    def __init__(self, B, feats, contents, mode, override, timestamp, max_length):
        self.B = B
        self.feats = feats
        self.streams = [_Stream(content_frames=c) for c in contents]
        self.left = sum(1 for s in self.streams if s.active)
        self.mode, self.override, self.timestamp = mode, override, timestamp
        self.pres = None
        self.host_stats = None
        self.gates = [(False, False, 0.0, 0.0, 0.0, 0.0, 0, 0)] * B
        self.tokens = np.full((B, max_length), -1, np.int32)   # first windows, with prompt
        self.n_tokens = np.zeros(B, np.int32)


@dataclasses.dataclass
class _Window:
    """One window of one clip waiting for, or riding in, the decoder."""
    batch: _Batch
    u: int            # clip index in its batch
    seek: int
    size: int
    prompt: list
    key: tuple        # (utterance, window counter): the fallback's noise seeds
    enc: object = None   # its encoder output: row `erow` of this fp16 [n][1500][d] tensor
    erow: int = 0


def _window(batch, u, tk, max_length):
    s = batch.streams[u]
    return _Window(batch, u, s.seek, s.window_size(), s.prompt(tk, max_length), (u, s.windows))


class PacketRenderer:
    """The decode side alone (engine.py:220-286 -> synthesizer.py:106-203): packets ->
    prompts -> front end -> Firefly-GAN vocoder, in the receiver's voice. ``weights``: the
    vocoder's tensors (default: JANUS_VOCODER_DIR or the seeded synthetic ones)."""

    def __init__(self, vocoder_cfg: FireflyConfig = FireflyConfig(), vocoder_seed: int = 0,
                 vocoder_weights: dict = None):
        self.device = nat.require_gpu()
        self.vocoder = VocoderEngine(vocoder_cfg, weights=vocoder_weights, seed=vocoder_seed)

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
        if getattr(self, "_stock_voice", None) is None or self._stock_for is not v:
            self._stock_voice = v.voice(DEFAULT_REFERENCE_ID)
            self._stock_for = v
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
        """The second vocoder context (the primary one's weights, its own workspaces) that
        renders the decoder side's share of a staggered step's batch; rebuilt when the
        primary engine is replaced."""
        if getattr(self, "_voc2", None) is None or self._voc2_of is not self.vocoder:
            v = self.vocoder
            self._voc2 = VocoderEngine(v.cfg, weights=v.weights)
            self._voc2_of = v
        return self._voc2


class JanusPipeline(PacketRenderer):
    def __init__(self, model: str = "base.en", whisper_seed: int = 0, vocoder_seed: int = 0,
                 max_length: int = 448, vocoder_cfg: FireflyConfig = FireflyConfig(),
                 temperatures=TEMPERATURES, tuning: Optional[ServingTuning] = None,
                 vocoder_weights: dict = None):
        """temperatures: faster-whisper's fallback schedule (the default, as the
        reference's transcribe_buffer runs it); (0.0,) decodes each window once at T = 0
        and only reports the gates (bench.py's headline setting on synthetic weights,
        whose windows all fail the gates: DESIGN.md §0)."""
        super().__init__(vocoder_cfg, vocoder_seed, vocoder_weights)
        self.whisper = WhisperEngine(CONFIGS[model], seed=whisper_seed)
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

    # ------------------------------------------------------------------ features
    def _features(self, pcm, offsets, lengths):
        """Whole-clip log-mel of every clip's [::3] (faster-whisper's one FeatureExtractor
        call per transcribe, normalised over all of the clip's frames), fp16 [B][F][80] with
        F = max(3000, the longest clip's content frames), zeros past each clip's content; and
        the first windows' mel [B][3000][80] (a view when F = 3000)."""
        B = len(lengths)
        cont = contents_of(lengths)
        F = max(N_FRAMES, max(cont) if cont else 0)
        w = self.whisper
        if F == N_FRAMES:
            feats = w.logmel(pcm, offsets, B, 3)
            return feats, feats, cont
        feats = w.logmel_frames(pcm, offsets, B, 3, F)
        return feats, feats[:, :N_FRAMES].contiguous(), cont

    def _seek_loop(self, feats, contents, enc1, dec1, **dec_kw):
        """faster-whisper's seek loop (generate_segments, transcriber.py:53-57) over one batch
        whose first windows are already decoded (dec1: T = 0 rows of enc1): the first round's
        gates and fallback, then rounds of continuation windows (their features sliced out of
        ``feats`` at each clip's seek, encoded, decoded with the <|startofprev|> prompt) until
        every clip's seek has reached its content. Host-driven, on the current stream. Returns
        (streams, first-window gates)."""
        w, L, tk = self.whisper, self.max_length, self.whisper.tokenizer
        B = len(contents)
        streams = [_Stream(content_frames=c) for c in contents]
        gates = [(False, False, 0.0, 0.0, 0.0, 0.0, 0, 0)] * B
        rows1 = dec1.rows()
        nt1 = dec1.n_tokens.cpu().numpy()
        first_round = True
        while True:
            act = [u for u in range(B) if streams[u].active]
            if not act:
                break
            for c0 in range(0, len(act), 64):
                idx = act[c0:c0 + 64]
                grp = [streams[u] for u in idx]
                sizes = [s.window_size() for s in grp]
                prompts = [s.prompt(tk, L) for s in grp]
                keys = [(u, s.windows) for u, s in zip(idx, grp)]
                if first_round:
                    enc, rows, nts, erows = enc1, [rows1[u] for u in idx], [nt1[u] for u in idx], idx
                else:
                    mel = gather_windows([(feats, u, s.seek, z) for u, s, z in zip(idx, grp, sizes)])
                    enc = w.encode(mel)
                    out = w.decode_ex(enc, prompts=prompts, max_length=L, **dec_kw)
                    rows, nts, erows = out.rows(), out.n_tokens.cpu().numpy(), None
                first, final, ndec = settle_round(w, tk, rows, prompts, keys, enc, L, self.temperatures,
                                                  BEST_OF, enc_rows=erows, **dec_kw)
                for u, s, z, c0r, r, nd, nt in zip(idx, grp, sizes, first, final, ndec, nts):
                    advance(tk, s, z, c0r, r, nd, nt)
                    if first_round:
                        gates[u] = _gates(c0r, r, nd, s)
                    if not self.tuning.all_windows:
                        s.seek = max(s.seek, s.content_frames)
            first_round = False
        return streams, gates

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
            feats, mel, cont = self._features(pcm, offsets, lengths)
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
            streams, gts = self._seek_loop(feats, cont, enc, dec)
        main.wait_stream(hi)
        tags = _tags(pres, None, B)
        return self._result(streams, gts, tags, pres, B, dec.tokens.cpu(), dec.n_tokens.cpu(), mode,
                            override, timestamp, pcm.device)

    def _result(self, streams, gates, tags, pres, B, tokens, n_tokens, mode, override, timestamp, dev):
        texts = [s.transcript() for s in streams]
        ts = time.time() if timestamp is None else timestamp
        packets = [JanusPacket(t, mode, g, override, ts).serialize() if t.strip() else None
                   for t, g in zip(texts, tags)]
        parts = pres if isinstance(pres, tuple) else (pres,)
        stats = _prosody_stats(parts if pres is not None else None, B, dev)
        return EncodeResult(texts, tags, packets, tokens, n_tokens, stats, gates, streams)

    def _xsplits(self, default):
        x = self.tuning.xattn_splits
        return default if x is None else x

    def _hi_stream(self, device):
        if getattr(self, "_hi", None) is None:
            self._hi = torch.cuda.Stream(device=device, priority=-1)
        return self._hi

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
        return self._dec_s.stream, self._voc_s.stream

    def step_overlapped(self, pcm, offsets, lengths, frames, dec_per_xcd: int = 16,
                        mode=JanusMode.SEMANTIC_VOICE, override="auto", timestamp=None):
        """One serving step of a two-stage pipeline: batch i goes through mel, encoder,
        greedy decoder and YIN; batch i-1 (kept from the previous call) through
        detokenisation, packets and the vocoder. Returns (EncodeResult, wav, pcm16) of batch
        i-1 — (None, None, None) on the first call; `flush` returns the last batch.

        Mel + encoder (compute-bound) get the whole GPU, and the host finishes batch i-1
        (transcripts, tags, MessagePack packets: a few ms) while they run. Then the greedy
        decoder of batch i's first windows (latency-bound) runs on a CU-masked stream holding
        `dec_per_xcd` CUs of each XCD, and the vocoder of batch i-1 followed by batch i's
        YIN on the disjoint rest, so neither holds the CUs the other needs (an unmasked
        overlap measured slower: the vocoder's long-running blocks delay every decoder
        launch). The rest of the seek loop (the fallback of failing windows, then the
        continuation windows) runs host-driven after both sides, on the whole GPU."""
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
        # after the decoder, to even out the two sides (r02-r03 sweeps: DESIGN.md §5b)
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
            feats, mel, cont = self._features(pcm, offsets, lengths)
            enc = w.encode(mel)
        if self.keep_encoder_output:   # [B][1500][d] fp16 of batch i, for parity checks only
            self.last_encoder_output = enc
        # batch i-1 on the host while the encoder runs (its tensors were joined into the
        # caller's stream at the end of the previous call)
        prev = getattr(self, "_pending", None)
        self._pending = None
        res_prev = self._finish(*prev) if prev is not None else None
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
            dec_kw = dict(xattn_splits=self._xsplits(4), cu_count=self._dec_s.n_cus)
            dec = w.decode_ex(enc, max_length=self.max_length, **dec_kw)
            if n_dec > 0:
                pres = (yin(0, n_dec), pres)
        # the rest of the seek loop (host-driven: reads the T = 0 tokens and gates): the
        # fallback's sampled re-decodes and the continuation windows, on the WHOLE GPU (the
        # high-priority stream, after the vocoder side and the first-window decode; the
        # 320-row cross-attention streams scale with the CUs; tuning.fallback_full False:
        # on the decoder's CUs)
        if self.tuning.fallback_full:
            hi.wait_stream(ds)
            hi.wait_stream(vs)
            fb_kw = dict(xattn_splits=self.tuning.fallback_xattn_splits,
                         cu_count=torch.cuda.get_device_properties(pcm.device).multi_processor_count)
            with torch.cuda.stream(hi):
                dec.settled = self._seek_loop(feats, cont, enc, dec, **fb_kw)
            ds.wait_stream(hi)
        else:
            with torch.cuda.stream(ds):
                dec.settled = self._seek_loop(feats, cont, enc, dec, **dec_kw)
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
        """Host tail of an overlapped step's batch: prosody tags (fallback Normal/Normal,
        engine.py:520-525), transcripts of the settled seek loop, packets (engine.py:527-548)."""
        tags = _tags(pres, None, B)
        streams, gts = dec.settled
        return self._result(streams, gts, tags, pres, B, dec.tokens.cpu(), dec.n_tokens.cpu(), mode,
                            override, timestamp, dec.tokens.device)

    def flush(self, frames):
        """Finish and render the batch the last overlapped step left pending:
        (EncodeResult, wav, pcm16), or (None, None, None)."""
        prev, self._pending = getattr(self, "_pending", None), None
        if prev is None:
            return None, None, None
        res = self._finish(*prev)
        wav, pcm16, _ = self.decode(res.packets, frames)
        return res, wav, pcm16

    # ------------------------------------------- staggered (continuous-batching) step
    def _prefetch(self, tensors, stream, key):
        """Device-to-host copies of ``tensors`` into pinned buffers (set ``key``), on a
        torch-owned stream behind ``stream``: the host tail then waits for the work that
        produced them alone, not — through the caller's stream — for the vocoder side that
        ends later. Returns (event, host tensors). One buffer set per key: the next copies
        into it are enqueued after the host tail has read these (the next step)."""
        hb = self._stag.setdefault("hbuf", {})
        cs = getattr(self, "_d2h_stream", None)
        if cs is None:
            cs = self._d2h_stream = torch.cuda.Stream(tensors[0].device)
        cs.wait_stream(stream)
        out = []
        with torch.cuda.stream(cs):
            for i, t in enumerate(tensors):
                t.record_stream(cs)   # the source outlives the copy (its allocator block)
                name = (key, i)
                buf = hb.get(name)
                if buf is None or buf.shape != t.shape or buf.dtype != t.dtype:
                    buf = hb[name] = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                buf.copy_(t, non_blocking=True)
                out.append(buf)
            ev = torch.cuda.Event()
            ev.record(cs)
        return ev, out

    def _stag_state(self, B, dev):
        st = getattr(self, "_stag", None)
        if st is not None and st["B"] != B:
            # the slot layout (and every KV / token row in it) is sized by B: windows still
            # in the decoder would be lost
            if self._stag_busy(st):
                raise ValueError(f"step_staggered: batch size {B} != {st['B']} while batches are "
                                 "in flight; call flush_staggered() first (or pad the batch)")
            st = None
        if st is None:
            n = max(2, self.tuning.stagger_sets)
            d = self.whisper.cfg.d_model
            R = B * self.tuning.batches_per_set()
            st = self._stag = {"B": B, "R": R, "n": n, "k": 0, "sets": [None] * n, "pos": [0] * n,
                               "started": False, "queue": collections.deque(), "completed": [],
                               "ready": collections.deque(),
                               "serial": 0,
                               "finished": collections.deque(), "calls": self.tuning.calls(),
                               "enc": torch.zeros(n * R, self.whisper.cfg.n_audio_ctx, d,
                                                  dtype=torch.float16, device=dev)}
        return st

    @staticmethod
    def _stag_busy(st):
        return (any(x is not None for x in st["sets"]) or st["queue"] or st["ready"]
                or st["completed"] or st["finished"])

    def staggered_depth(self):
        """Steps before the first batch comes out when every clip has two windows (30 s clips
        on the synthetic weights): a window group completes N - 1 calls after it entered and
        is absorbed at the next step; with all windows the continuation windows enter in the
        step that absorbed the first ones (one call per step: 2N; two calls per step, the
        second taking them: N + 1); first windows only: N."""
        n = max(2, self.tuning.stagger_sets)
        if not self.tuning.all_windows:
            return n
        late = 1 if self.tuning.cont_encode == "voc" else 0   # encoded a step before entering
        return (2 * n if self.tuning.calls() == 1 else n + 1) + late

    def _absorb(self, st):
        """Host part of the windows the previous step's decoder calls completed: each
        window's gates (and, with the fallback on, its sampled re-decodes on the whole GPU in
        decoder state slot 1), the seek-loop update of its clip (segments, next seek,
        prompt), a continuation window queued for every clip whose seek is still short of its
        content, and every batch whose clips are all done moved to ``finished``."""
        comp, st["completed"] = st["completed"], []
        if not comp:
            return
        w, L, tk = self.whisper, self.max_length, self.whisper.tokenizer
        fb_kw = dict(xattn_splits=self.tuning.fallback_xattn_splits,
                     cu_count=torch.cuda.get_device_properties(self.device).multi_processor_count,
                     state_slot=1)
        for rec, host in comp:
            ev, (tok, nt, lp, ns) = host
            if ev is not None:
                ev.synchronize()
            else:   # tuning.host_prefetch off: read the device rows (waits for their stream)
                tok, nt, lp, ns = (t.cpu() for t in (tok, nt, lp, ns))
            # the staggered calls do not wait for their stream (check_every 0): their
            # persistent grids' barrier-timeout flag is read here, before the rows are used
            w.decode_check()
            items, plens = rec["items"], rec["plens"]
            tok, nt, lp, ns = tok.numpy(), nt.numpy(), lp.numpy(), ns.numpy()
            rows = []
            eot = w.tokenizer.eot
            for j in range(len(items)):
                s = tok[j][int(plens[j]):int(plens[j]) + int(nt[j])]
                s = s[s != eot].tolist()
                rows.append((s, float(lp[j]) / (len(s) + 1), float(ns[j])))
            prompts = [it.prompt for it in items]
            keys = [it.key for it in items]
            with torch.cuda.stream(self._hi_stream(self.device)):   # re-decodes: whole GPU
                enc = (torch.cat([t[r0:r0 + c] for t, r0, c in rec["enc"]])
                       if len(self.temperatures) > 1 else None)
                first, final, ndec = settle_round(w, tk, rows, prompts, keys, enc, L,
                                                  self.temperatures, BEST_OF, **fb_kw)
            for j, (it, c0, r, nd) in enumerate(zip(items, first, final, ndec)):
                b, s = it.batch, it.batch.streams[it.u]
                was_first = s.windows == 0
                advance(tk, s, it.size, c0, r, nd, nt[j])
                if was_first:
                    b.gates[it.u] = _gates(c0, r, nd, s)
                    b.tokens[it.u] = tok[j][:L]
                    b.n_tokens[it.u] = nt[j]
                    if not self.tuning.all_windows:
                        s.seek = max(s.seek, s.content_frames)
                if s.active:
                    st["queue"].append(_window(b, it.u, tk, L))
                else:
                    b.left -= 1
                    if b.left == 0:
                        st["finished"].append(b)
        # a batch finishes when its last clip does (the queue order keeps them in order
        # whenever every clip takes the same number of windows)

    def _finish_batch(self, b) -> EncodeResult:
        """Host tail of a finished batch: tags, transcripts (each clip's segments joined),
        packets."""
        tags = _tags(b.pres, b.host_stats, b.B)
        b.feats = None
        return self._result(b.streams, b.gates, tags, b.pres, b.B, torch.from_numpy(b.tokens),
                            torch.from_numpy(b.n_tokens), b.mode, b.override, b.timestamp,
                            self.device)

    def step_staggered(self, pcm, offsets, lengths, frames, dec_per_xcd: int = 16,
                       mode=JanusMode.SEMANTIC_VOICE, override="auto", timestamp=None):
        """The serving step with the greedy decoder as a continuous batch of WINDOWS: every
        decoder call advances N slot sets of B rows (N = tuning.stagger_sets) by S =
        ceil((max_length - 1) / N) positions (janus_decode_rows.pos_offset); one set takes a
        fresh group of up to B windows, the set that entered N - 1 calls earlier completes.
        A window is one 30 s Whisper window of one clip: the first windows of a new batch,
        and the continuation windows faster-whisper's seek loop decodes from the seek the
        previous window ended at (transcriber.py:53-57: its features sliced out of the clip's
        whole log-mel, zero-padded, its prompt <|startofprev|> + the clip's last 223 tokens)
        — they re-enter the continuous batch as new rows. Per step:

          host      the windows completed by the previous step's calls: gates (and the
                    fallback's re-decodes, whole GPU, decoder state slot 1), the seek loop
                    of their clips, continuation windows queued, finished batches
          hi        log-mel of batch i, the encoder of its first windows, then the encoder
                    of the queued continuation windows (whole GPU)
          decoder   tuning.calls() calls (2 with all windows): the first windows of batch i
          CUs       enter in the first, the oldest queued continuation windows in the next;
                    YIN of the first n_dec utterances of batch i beside them (_yin_split)
          vocoder   the oldest finished batch, then the rest of batch i's YIN
          CUs

        so that with two windows per clip every step takes in one batch, decodes 2B windows
        and renders one batch. Returns (EncodeResult, wav, pcm16) of the batch rendered,
        (None, None, None) while the pipeline fills; ``flush_staggered`` drains. Per-row
        results are bit-identical to the one-batch decode (rows are independent of their
        neighbours' positions), so each clip's transcript is the seek loop's."""
        B = len(lengths)
        w = self.whisper
        L = self.max_length
        tk = w.tokenizer
        dev = pcm.device if pcm is not None else self.device
        main = torch.cuda.current_stream(dev)
        hi = self._hi_stream(dev)
        ds, vs = self._split_streams(dev, dec_per_xcd)
        st = self._stag_state(B, dev)
        n, C = st["n"], st["calls"]
        # S positions per call cover the full decode's L - 1 steps in N calls; the last set's
        # chunk may overrun by a position (a no-op past the row's end) but not past L
        S = -(-(L - 1) // n)
        if n * S > L:
            raise ValueError(f"stagger_sets={n} does not tile max_length {L}")
        hi.wait_stream(main)
        nb = None
        enc1 = None
        if pcm is not None:
            with torch.cuda.stream(hi):
                feats, mel, cont = self._features(pcm, offsets, lengths)
                enc1 = w.encode(mel)
            nb = _Batch(B, feats, cont, mode, override, timestamp, L)
            nb.serial = st["serial"]
            st["serial"] += 1
        # the windows the previous step completed, on the host while the encoder runs
        self._absorb(st)
        # this step's groups: the new batch's first windows, then the continuation windows,
        # oldest first — with cont_encode "voc" those encoded on the vocoder's CUs during the
        # previous step (st["ready"]), with "hi" the queued ones, encoded below on the whole GPU
        pend = ([_Window(nb, u, 0, nb.streams[u].window_size(), list(tk.sot_sequence), (u, 0), enc1, u)
                 for u in range(B) if nb.streams[u].active] if nb is not None else [])
        late = self.tuning.cont_encode == "voc"
        src_q = st["ready"] if late else st["queue"]
        pend += list(src_q)
        src_q.clear()
        R = st["R"]
        groups = []
        for c in range(C):
            g, pend = pend[:R], pend[R:]
            groups.append(g if g else None)
        src_q.extend(pend)
        if not late:
            # the groups' continuation windows encoded here from their clips' features (one
            # encoder call on the whole GPU, before the decoder call)
            conts = [it for g in groups if g for it in g if it.enc is None]
            with torch.cuda.stream(hi):
                if conts:
                    mel2 = gather_windows([(it.batch.feats, it.u, it.seek, it.size) for it in conts])
                    enc2 = w.encode(mel2)
                    for i, it in enumerate(conts):
                        it.enc, it.erow = enc2, i
        # each group's encoder rows as runs of consecutive rows of the windows' encoder
        # outputs [(tensor, first row, rows)], copied straight into the slot set's rows by its call
        gencs = []
        for g in groups:
            runs = []
            for it in g or []:
                src, r = it.enc, it.erow
                if runs and runs[-1][0] is src and runs[-1][1] + runs[-1][2] == r:
                    runs[-1][2] += 1
                else:
                    runs.append([src, r, 1])
            gencs.append(runs if g else None)
        if self.keep_encoder_output:   # parity checks: every window's encoder rows and inputs
            log = self.__dict__.setdefault("window_log", {})
            for g, runs in zip(groups, gencs):
                rows = [t[r0 + i] for t, r0, c in (runs or []) for i in range(c)]
                for it, e in zip(g or [], rows):
                    log[(it.batch.serial, it.u, it.key[1])] = (e, list(it.prompt), it.seek, it.size)
        # the oldest finished batch on the host (its windows all settled)
        fin = st["finished"].popleft() if st["finished"] else None
        res_prev = self._finish_batch(fin) if fin is not None else None
        vs.wait_stream(hi)
        ds.wait_stream(hi)
        record = getattr(self, "side_events", None) is not None
        # side events every step: the YIN split below reads the previous step's
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record(vs)
        ev[2].record(ds)
        wav = pcm16 = None
        pres = None
        # YIN of the first n_dec utterances runs on the decoder side (beside the decoder calls,
        # below), the rest behind the vocoder
        n_dec = self._yin_split(st, B) if pcm is not None else 0

        def yin(u0, u1):
            try:
                return prosody_launch(pcm, offsets[u0:u1 + 1], lengths[u0:u1], CAPTURE_RATE, 512,
                                      max_blocks=0)
            except Exception:  # engine.py:520-525
                return None
        # the last kv packets of the rendered batch on the decoder's CUs after its calls (a
        # second vocoder context), the rest here (tuning.voc_dec_utts)
        kv = 0
        pk_dec = []
        wav_b = pcm_b = None
        with torch.cuda.stream(vs):
            if late and st["queue"]:
                # the continuation windows queued by this step's host part, encoded on the
                # vocoder's CUs (its side has the slack): they enter the next step's call
                todo = list(st["queue"])
                st["queue"].clear()
                mel2 = gather_windows([(it.batch.feats, it.u, it.seek, it.size) for it in todo])
                enc2 = w.encode(mel2)
                for i, it in enumerate(todo):
                    it.enc, it.erow = enc2, i
                st["ready"].extend(todo)
            if res_prev is not None:
                pk = res_prev.packets
                kv = min(len(pk), max(0, self.tuning.voc_dec_utts))
                self.voc_dec_utts = kv   # the main vocoder context renders the other len(pk) - kv
                pk_dec = pk[len(pk) - kv:] if kv else []
                wav, pcm16, _ = self.decode(pk[:len(pk) - kv], frames)
            if pcm is not None:
                pres = yin(n_dec, B)
            ev[1].record(vs)
        busy = any(g is not None for g in groups) or any(x is not None for x in st["sets"])
        if busy:
            with torch.cuda.stream(ds):
                # the decoder side's YIN runs concurrently with the decode calls, on a second
                # stream over the decoder's CUs with its grid capped at tuning.yin_beside blocks
                # (default 128; 0: after the calls): the latency-bound decoder leaves issue
                # slots free (profiles/r04_yin_beside_ab.json)
                # (not beside a 256-row call: its resident grid holds two blocks on every
                # CU of the partition, the YIN blocks would keep them from co-residing)
                yb = self.tuning.yin_beside
                beside = yb > 0 and n_dec > 0 and st["n"] * st["R"] <= 128
                if beside:
                    ys = self._yin_s.stream
                    ys.wait_stream(ds)
                    with torch.cuda.stream(ys):
                        try:
                            pd = prosody_launch(pcm, offsets[0:n_dec + 1], lengths[0:n_dec], CAPTURE_RATE,
                                                512, max_blocks=yb)
                        except Exception:  # engine.py:520-525
                            pd = None
                for c in range(C):
                    g = groups[c]
                    if g is None and not any(x is not None for x in st["sets"]):
                        continue
                    self._stag_call(st, g, gencs[c], S, c)
                if beside:
                    ds.wait_stream(ys)
                    pres = (pd, pres)
                elif n_dec > 0:
                    pres = (yin(0, n_dec), pres)
        elif pcm is not None and n_dec > 0:
            with torch.cuda.stream(ds):
                pres = (yin(0, n_dec), pres)
        if pk_dec:
            with torch.cuda.stream(ds):
                wav_b, pcm_b, _ = self.decode(pk_dec, frames, vocoder=self._vocoder_dec())
        if nb is not None:
            nb.pres = pres
            parts = pres if isinstance(pres, tuple) else (pres,)
            if all(p is not None for p in parts):
                # the batch's YIN statistics, copied behind both YIN launches (read when the
                # batch finishes, steps later)
                cs = getattr(self, "_d2h_stream", None)
                if cs is None:
                    cs = self._d2h_stream = torch.cuda.Stream(dev)
                cs.wait_stream(ds)
                cs.wait_stream(vs)
                with torch.cuda.stream(cs):
                    hp = [tuple(torch.empty(t.shape, dtype=t.dtype, pin_memory=True).copy_(t, non_blocking=True)
                                for t in (p.rms, p.mean_f0, p.n_voiced)) for p in parts]
                    e = torch.cuda.Event()
                    e.record(cs)
                nb.host_stats = (e, hp)
        ev[3].record(ds)
        if record:
            self.side_events.append(ev)
        # only full steps (a vocoder batch, a batch entering) steer the YIN split
        if pcm is not None and res_prev is not None and busy:
            st["prev_ev"] = ev
        main.wait_stream(ds)
        main.wait_stream(vs)
        if wav_b is not None:   # the batch back in packet order
            wav = wav_b if wav is None else torch.cat([wav, wav_b])
            pcm16 = pcm_b if pcm16 is None else torch.cat([pcm16, pcm_b])
        return res_prev, wav, pcm16

    def _stag_call(self, st, g, runs, S, c):
        """One staggered decoder call on the current (decoder) stream: group ``g`` (a list of
        windows, or None) enters the fresh slot set (its encoder rows copied into the set's
        rows of the call's encoder buffer; its prompts), every other set continues; the set
        whose group completes gets its results copied to the host behind the call."""
        w, L, tk = self.whisper, self.max_length, self.whisper.tokenizer
        B, n = st["R"], st["n"]     # rows per slot set
        k = st["k"]
        f = k % n
        ds = torch.cuda.current_stream()
        if g is not None:
            o = f * B
            for t, r0, cnt in runs:
                st["enc"][o:o + cnt].copy_(t[r0:r0 + cnt])
                o += cnt
        pos = st["pos"]
        set_offs, jc = stagger_plan(st["sets"], pos, st["started"], k, S, g is not None)
        offs = [o for o in set_offs for _ in range(B)]
        sot = list(tk.sot_sequence)
        prompts = [sot] * (n * B)
        if g is not None:
            for j, it in enumerate(g):
                prompts[f * B + j] = it.prompt
        lgb = self.tuning.logits_blocks
        if lgb <= 0:   # one round: the decoder's CUs over the call's 64-row groups
            lgb = max(8, (self._dec_s.n_cus // ((n * B + 63) // 64)) // 8 * 8)
        dec = w.decode_ex(st["enc"], prompts=prompts, max_length=L, pos_offset=offs, steps=S,
                          xattn_splits=self._xsplits(1), cu_count=self._dec_s.n_cus,
                          persistent=self.tuning.persistent, path_flags=self.tuning.dec_path_flags,
                          logits_blocks=lgb, check_every=self.tuning.dec_poll)
        st["started"] = True
        # where each set's rows stand now (offset + S, or fewer when every row finished and
        # the call stopped early), as the context recorded it
        stand = w.decode_stand(n * B)
        for j in range(n):
            pos[j] = stand[j * B]
        if jc is not None:
            rec = st["sets"][jc]
            m = len(rec["items"])
            sl = slice(jc * B, jc * B + m)
            parts = [dec.tokens[sl], dec.n_tokens[sl], dec.sum_logprob[sl], dec.no_speech_prob[sl]]
            host = self._prefetch(parts, ds, c) if self.tuning.host_prefetch else (None, parts)
            st["completed"].append((rec, host))
            st["sets"][jc] = None
        if g is not None:
            st["sets"][f] = {"born": k, "items": g, "plens": [len(it.prompt) for it in g],
                             "enc": runs}
        st["k"] = k + 1

    # YIN of one 30 s utterance on a 16-CU-per-XCD partition (26 ms for 64, either side)
    YIN_MS_PER_UTT = 0.4

    def _yin_split(self, st, B):
        """Utterances whose YIN runs on the decoder side in the staggered step. Fixed by
        tuning.yin_dec_utts; otherwise self-balancing: starts at 7B/8 (where it settled on
        the r04 boxes: 52-59 of 64) when the decoder call leaves room for YIN beside it (at
        most 128 rows), at 0 when it does not (every window decoded: 256 rows, the decoder
        side binds and YIN after its call would lengthen it — r06 traces showed the 7B/8
        start needing four steps to walk down), and moves by the previous full step's side-time gap
        (vocoder side minus decoder side, HIP events on the two CU-masked streams) over
        twice the per-utterance YIN time, at most 16 per step,
        so the two partitions finish together whatever the box's vocoder / decoder speed
        ratio (measured from box to box: vocoder side 253-265 ms at the same split)."""
        if self.tuning.yin_dec_utts is not None:
            return max(0, min(B - 1, self.tuning.yin_dec_utts))
        n = st.get("n_dec", 7 * B // 8 if st["n"] * st["R"] <= 128 else 0)
        prev = st.get("prev_ev")
        if prev is not None and prev[1].query() and prev[3].query():
            gap = prev[0].elapsed_time(prev[1]) - prev[2].elapsed_time(prev[3])
            move = int(round(gap / (2.0 * self.YIN_MS_PER_UTT)))
            n = max(0, min(B - 1, n + max(-16, min(16, move))))
        st["n_dec"] = n
        return n

    def flush_staggered(self, frames):
        """Drain the staggered pipeline: decode every window still queued or in the decoder
        and render the batches. Returns a list of (EncodeResult, wav, pcm16), in order."""
        out = []
        st = getattr(self, "_stag", None)
        if st is None:
            return out
        while self._stag_busy(st):
            r = self.step_staggered(None, None, [0] * st["B"], frames)
            if r[0] is not None:
                out.append(r)
        self._stag = None
        return out


def _gates(c0, r, nd, s):
    """The first window's gates as EncodeResult.gates holds them (after advance)."""
    skip = r.no_speech_prob > 0.6 and not r.avg_logprob > -1.0
    return (c0.needs_fallback, skip, r.avg_logprob, r.compression_ratio, r.no_speech_prob,
            r.temperature, nd, s.seek)
