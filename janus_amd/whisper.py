"""Whisper model host side: configs, weights, front-end constants and the GPU engine.

The engine owns one ``janus_whisper`` context (include/janus.h) and calls
``janus_whisper_logmel`` -> ``janus_whisper_encode`` -> ``janus_whisper_decode_greedy``
on torch-allocated device buffers and torch's current stream.

Weights: if ``JANUS_WHISPER_DIR`` points at a Hugging Face Whisper checkpoint
(``model.safetensors``), it is loaded (safetensors, no pickle). Otherwise the model has
seeded synthetic weights of the real shapes (no checkpoints are reachable offline).
"""
import ctypes
import dataclasses
import math
import os

import numpy as np
import torch

from . import _native as nat
from . import tokenizer as tok


@dataclasses.dataclass(frozen=True)
class WhisperConfig:
    name: str
    d_model: int
    n_heads: int
    enc_layers: int
    dec_layers: int
    n_mels: int = 80
    n_audio_ctx: int = 1500
    n_vocab: int = tok.N_VOCAB_EN
    n_text_ctx: int = 448

    @property
    def ffn(self):
        return 4 * self.d_model


CONFIGS = {
    "tiny.en": WhisperConfig("tiny.en", 384, 6, 4, 4),
    "base.en": WhisperConfig("base.en", 512, 8, 6, 6),
    "small.en": WhisperConfig("small.en", 768, 12, 12, 12),
}


class janus_whisper_config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("n_mels", "n_audio_ctx", "d_model", "n_heads",
                                            "enc_layers", "dec_layers", "n_vocab", "n_text_ctx")]


class janus_decode_options(ctypes.Structure):
    _fields_ = [("prompt", ctypes.POINTER(ctypes.c_int32)), ("prompt_len", ctypes.c_int),
                ("max_length", ctypes.c_int), ("eot", ctypes.c_int),
                ("suppress", ctypes.POINTER(ctypes.c_int32)), ("n_suppress", ctypes.c_int),
                ("suppress_blank", ctypes.c_int), ("blank_token", ctypes.c_int),
                ("timestamp_begin", ctypes.c_int), ("no_timestamps", ctypes.c_int),
                ("max_initial_timestamp_index", ctypes.c_int), ("check_every", ctypes.c_int),
                ("xattn_splits", ctypes.c_int), ("cu_count", ctypes.c_int),
                ("state_slot", ctypes.c_int), ("logits_blocks", ctypes.c_int),
                ("msplit_rows_n", ctypes.c_int), ("persistent", ctypes.c_int),
                ("path_flags", ctypes.c_uint32), ("lanes", ctypes.c_int)]


# janus_decode_options.path_flags (include/janus.h JANUS_DEC_PATH_*): alternative decoder
# paths the parity tests hold bit-identical to the default; 0 = the measured default
DEC_PATH_NO_GRAPH = 0x0001
DEC_PATH_NO_XABSORB = 0x0002
DEC_PATH_NO_XPAIR = 0x0004
DEC_PATH_XGROUP = 0x0008
DEC_PATH_FUSED_LN = 0x0010
DEC_PATH_LN_FUSE = 0x0020
DEC_PATH_RESID_LN = 0x0040
DEC_PATH_NO_CVP = 0x0080
DEC_PATH_CVP = 0x0100
DEC_PATH_NO_SEL_EMBED = 0x0200
DEC_PATH_NO_EMBED_LN = 0x0400
DEC_PATH_LN_PROLOGUE = 0x0800
DEC_PATH_SEG_2CU = 0x10000
DEC_PATH_XFWD = 0x20000


def dec_path_ln_mask(m: int) -> int:
    """JANUS_DEC_PATH_LN_MASK(m): LayerNorm-into-prologue mask m instead of the default."""
    return DEC_PATH_LN_PROLOGUE | ((m & 15) << 12)


class janus_decode_rows(ctypes.Structure):
    _fields_ = [("prompts", ctypes.POINTER(ctypes.c_int32)),
                ("prompt_lens", ctypes.POINTER(ctypes.c_int32)),
                ("stride", ctypes.c_int), ("no_speech_token", ctypes.c_int),
                ("enc_index", ctypes.POINTER(ctypes.c_int32)), ("n_enc", ctypes.c_int),
                ("pos_offset", ctypes.POINTER(ctypes.c_int32)), ("steps", ctypes.c_int)]


# ----------------------------------------------------------------- front end
def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """Whisper's fixed encoder positional embedding (openai whisper model.sinusoids)."""
    inc = np.log(max_timescale) / (channels // 2 - 1)
    inv = np.exp(-inc * np.arange(channels // 2))
    t = np.arange(length)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], axis=1).astype(np.float32)


def hz_to_mel_slaney(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp, min_log_hz, min_log_mel, logstep = 200.0 / 3, 1000.0, 15.0, np.log(6.4) / 27.0
    mel = f / f_sp
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mel)


def mel_to_hz_slaney(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp, min_log_hz, min_log_mel, logstep = 200.0 / 3, 1000.0, 15.0, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filters(sr=16000, n_fft=400, n_mels=80, fmin=0.0, fmax=8000.0) -> np.ndarray:
    """Slaney-normalised, slaney-scale triangular mel filters, [n_fft//2+1][n_mels]
    (librosa.filters.mel(htk=False, norm='slaney'), as faster-whisper's get_mel_filters)."""
    fft_freqs = np.linspace(0, sr // 2, 1 + n_fft // 2)
    mel_pts = np.linspace(hz_to_mel_slaney(fmin), hz_to_mel_slaney(fmax), n_mels + 2)
    f_pts = mel_to_hz_slaney(mel_pts)
    fdiff = np.diff(f_pts)
    ramps = f_pts[:, None] - fft_freqs[None, :]
    w = np.zeros((n_mels, len(fft_freqs)))
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (f_pts[2:n_mels + 2] - f_pts[:n_mels])
    w *= enorm[:, None]
    return w.T.astype(np.float32)  # [201][80]


def mel_constants():
    """("mel.basis" [400][416], "mel.filters" [208][80]) for janus_whisper_set_tensor."""
    n = np.arange(400)
    hann = 0.5 - 0.5 * np.cos(2 * np.pi * n / 400)  # periodic (torch.hann_window / np.hanning(401)[:-1])
    k = np.arange(201)
    ang = 2 * np.pi * np.outer(n, k) / 400
    basis = np.zeros((400, 416))
    basis[:, :201] = hann[:, None] * np.cos(ang)
    basis[:, 208:208 + 201] = hann[:, None] * np.sin(ang)
    filt = np.zeros((208, 80), np.float32)
    filt[:201] = mel_filters()
    return basis.astype(np.float32), filt


# -------------------------------------------------------------------- weights
def synthetic_weights(cfg: WhisperConfig, seed: int = 0) -> dict:
    """Seeded fp32 weights of the real shapes, HF naming (no 'model.' prefix)."""
    g = torch.Generator().manual_seed(seed)
    d, ff = cfg.d_model, cfg.ffn
    W = {}

    def rn(name, *shape, std=0.02):
        W[name] = (torch.randn(*shape, generator=g) * std).numpy().astype(np.float32)

    def ln(name):
        W[name + ".weight"] = (1.0 + 0.1 * torch.randn(d, generator=g)).numpy().astype(np.float32)
        W[name + ".bias"] = (0.02 * torch.randn(d, generator=g)).numpy().astype(np.float32)

    rn("encoder.conv1.weight", d, cfg.n_mels, 3, std=1.0 / math.sqrt(cfg.n_mels * 3))
    rn("encoder.conv1.bias", d)
    rn("encoder.conv2.weight", d, d, 3, std=1.0 / math.sqrt(d * 3))
    rn("encoder.conv2.bias", d)
    W["encoder.embed_positions.weight"] = sinusoids(cfg.n_audio_ctx, d)

    def attn(p, cross=False):
        for n in ("q", "k", "v", "out"):
            rn(f"{p}.{n}_proj.weight", d, d, std=1.0 / math.sqrt(d))
            if n != "k":
                rn(f"{p}.{n}_proj.bias", d)

    def mlp(p):
        rn(f"{p}.fc1.weight", ff, d, std=1.0 / math.sqrt(d))
        rn(f"{p}.fc1.bias", ff)
        rn(f"{p}.fc2.weight", d, ff, std=1.0 / math.sqrt(ff))
        rn(f"{p}.fc2.bias", d)

    for i in range(cfg.enc_layers):
        p = f"encoder.layers.{i}"
        attn(p + ".self_attn")
        ln(p + ".self_attn_layer_norm")
        mlp(p)
        ln(p + ".final_layer_norm")
    ln("encoder.layer_norm")
    rn("decoder.embed_tokens.weight", cfg.n_vocab, d, std=0.05)
    rn("decoder.embed_positions.weight", cfg.n_text_ctx, d, std=0.02)
    for i in range(cfg.dec_layers):
        p = f"decoder.layers.{i}"
        attn(p + ".self_attn")
        ln(p + ".self_attn_layer_norm")
        attn(p + ".encoder_attn")
        ln(p + ".encoder_attn_layer_norm")
        mlp(p)
        ln(p + ".final_layer_norm")
    ln("decoder.layer_norm")
    return engine_weights(W)


# tensors the engine reads in fp32 (whisper.cpp: the decoder's positional table is added
# to the token embedding in fp32); every other matrix is stored fp16 on the GPU
FP32_MATRICES = frozenset({"decoder.embed_positions.weight"})


def engine_weights(W: dict) -> dict:
    """The numbers the engine multiplies: every matrix the GPU stores in fp16 (conv
    kernels, projections, the token embedding, the encoder's positional table; ndim >= 2)
    rounded to fp16, as a CTranslate2 float16 conversion stores them; biases, LayerNorm
    parameters and the fp32-consumed tables (FP32_MATRICES) stay fp32. The oracle is run on
    these weights, so parity measures arithmetic, not weight rounding."""
    return {k: (v.astype(np.float16).astype(np.float32) if v.ndim >= 2 and k not in FP32_MATRICES
                else v.astype(np.float32))
            for k, v in W.items()}


def load_weights(cfg: WhisperConfig, seed: int = 0) -> dict:
    """``JANUS_WHISPER_DIR/model.safetensors`` (a Hugging Face Whisper checkpoint: names
    ``model.encoder.*`` / ``model.decoder.*``, fp16 or fp32; ``proj_out.weight`` must be
    the tied token embedding) mapped to the engine's names, else seeded synthetic weights
    of the real shapes."""
    path = os.environ.get("JANUS_WHISPER_DIR")
    if path and os.path.exists(os.path.join(path, "model.safetensors")):
        from safetensors.numpy import load_file
        raw = load_file(os.path.join(path, "model.safetensors"))
        W = {k[len("model."):] if k.startswith("model.") else k: v for k, v in raw.items()}
        proj = W.pop("proj_out.weight", None)
        if proj is not None and not np.array_equal(proj, W.get("decoder.embed_tokens.weight")):
            raise ValueError("proj_out.weight differs from decoder.embed_tokens.weight: the "
                             "engine's vocabulary projection is the tied embedding")
        emb = W.get("decoder.embed_tokens.weight")
        if emb is None or emb.shape != (cfg.n_vocab, cfg.d_model):
            raise ValueError(f"checkpoint does not match {cfg.name}: decoder.embed_tokens.weight "
                             f"{None if emb is None else emb.shape}")
        return engine_weights(W)
    return synthetic_weights(cfg, seed)


# --------------------------------------------------------------------- engine
class WhisperEngine:
    """One janus_whisper context on the current GPU (thread-safe per call in C++)."""

    def __init__(self, cfg: WhisperConfig, weights: dict = None, seed: int = 0):
        self.device = nat.require_gpu()
        self.cfg = cfg
        self.tokenizer = tok.load_tokenizer()
        c = janus_whisper_config(cfg.n_mels, cfg.n_audio_ctx, cfg.d_model, cfg.n_heads,
                                 cfg.enc_layers, cfg.dec_layers, cfg.n_vocab, cfg.n_text_ctx)
        h = ctypes.c_void_p()
        nat.call("janus_whisper_create", ctypes.addressof(c), ctypes.addressof(h))
        self._h = h
        weights = weights if weights is not None else load_weights(cfg, seed)
        basis, filt = mel_constants()
        weights = dict(weights)
        weights["mel.basis"] = basis
        weights["mel.filters"] = filt
        for name, arr in weights.items():
            a = np.ascontiguousarray(arr, dtype=np.float32)
            nat.call("janus_whisper_set_tensor", self._h, name.encode(), a.ctypes.data, a.size)

    def set_tensor(self, name: str, arr) -> None:
        """Re-upload one parameter (janus_whisper_set_tensor); the next call re-prepares
        the derived fp16 weights and re-captures the decode graphs."""
        a = np.ascontiguousarray(arr, dtype=np.float32)
        nat.call("janus_whisper_set_tensor", self._h, name.encode(), a.ctypes.data, a.size)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                nat.lib().janus_whisper_destroy(h)
            except Exception:
                pass

    # ---- stages (device tensors in/out, current stream)
    def logmel(self, pcm: torch.Tensor, offsets: torch.Tensor, batch: int, decim: int,
               want_raw: bool = False):
        frames = 2 * self.cfg.n_audio_ctx
        mel = torch.empty(batch, frames, 80, dtype=torch.float16, device=self.device)
        raw = torch.empty(batch, frames, 80, dtype=torch.float32, device=self.device) if want_raw else None
        nat.call("janus_whisper_logmel", self._h, pcm.data_ptr(), offsets.data_ptr(), batch, decim,
                 raw.data_ptr() if raw is not None else None, mel.data_ptr(), nat.stream_ptr())
        return (mel, raw) if want_raw else mel

    def logmel_frames(self, pcm: torch.Tensor, offsets: torch.Tensor, batch: int, decim: int,
                      frames: int) -> torch.Tensor:
        """Whole-clip features (janus_whisper_logmel_frames): fp16 [batch][frames][80],
        normalised over every frame of each clip, 0.0 from each clip's content end on."""
        mel = torch.empty(batch, frames, 80, dtype=torch.float16, device=self.device)
        nat.call("janus_whisper_logmel_frames", self._h, pcm.data_ptr(), offsets.data_ptr(), batch,
                 decim, frames, mel.data_ptr(), nat.stream_ptr())
        return mel

    def encode(self, mel: torch.Tensor) -> torch.Tensor:
        B = mel.shape[0]
        assert mel.dtype == torch.float16 and mel.is_contiguous()
        enc = torch.empty(B, self.cfg.n_audio_ctx, self.cfg.d_model, dtype=torch.float16,
                          device=self.device)
        nat.call("janus_whisper_encode", self._h, mel.data_ptr(), B, enc.data_ptr(), nat.stream_ptr())
        return enc

    def decode_options(self, max_length: int = 448, check_every: int = 16,
                       timestamps: bool = True, xattn_splits: int = 0, cu_count: int = 0,
                       state_slot: int = 0, logits_blocks: int = 0, msplit_rows_n: int = 0,
                       persistent: int = 0, path_flags: int = 0, lanes: int = 0):
        t = self.tokenizer
        prompt = np.array(t.sot_sequence, np.int32)
        supp = np.array(t.suppress_tokens(), np.int32)
        opt = janus_decode_options()
        opt.prompt = prompt.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        opt.prompt_len = len(prompt)
        opt.max_length = max_length
        opt.eot = t.eot
        opt.suppress = supp.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        opt.n_suppress = len(supp)
        opt.suppress_blank = 1
        opt.blank_token = t.blank
        opt.timestamp_begin = t.timestamp_begin if timestamps else -1
        opt.no_timestamps = t.no_timestamps
        opt.max_initial_timestamp_index = 50
        opt.check_every = check_every
        opt.xattn_splits = xattn_splits
        opt.cu_count = cu_count
        opt.state_slot = state_slot
        opt.logits_blocks = logits_blocks
        opt.msplit_rows_n = msplit_rows_n
        opt.persistent = persistent
        opt.path_flags = path_flags
        opt.lanes = lanes
        return opt, (prompt, supp)

    def decode(self, enc: torch.Tensor, max_length: int = 448, check_every: int = 16,
               timestamps: bool = True, xattn_splits: int = 0, cu_count: int = 0,
               path_flags: int = 0, lanes: int = 0):
        B = enc.shape[0]
        opt, keep = self.decode_options(max_length, check_every, timestamps, xattn_splits,
                                        cu_count, path_flags=path_flags, lanes=lanes)
        tokens = torch.empty(B, max_length, dtype=torch.int32, device=self.device)
        ntok = torch.empty(B, dtype=torch.int32, device=self.device)
        slp = torch.empty(B, dtype=torch.float32, device=self.device)
        nat.call("janus_whisper_decode_greedy", self._h, enc.data_ptr(), B, ctypes.addressof(opt),
                 tokens.data_ptr(), ntok.data_ptr(), slp.data_ptr(), nat.stream_ptr())
        del keep
        return tokens, ntok, slp

    def decode_ex(self, enc: torch.Tensor, prompts=None, max_length: int = 448,
                  check_every: int = 16, timestamps: bool = True, xattn_splits: int = 0,
                  cu_count: int = 0, temperature: float = 0.0, seeds=None, enc_index=None,
                  pos_offset=None, steps: int = 0, state_slot: int = 0, logits_blocks: int = 0,
                  msplit_rows_n: int = 0, persistent: int = 0, path_flags: int = 0):
        """janus_whisper_decode_greedy_ex: per-row prompts (lists of token ids; None = the
        SOT sequence for every row) and the no-speech probability. Returns a DecodeOut.
        temperature > 0 samples instead (janus_whisper_decode_sample_ex: Gumbel-max over the
        rule-filtered logits / T with per-row uint32 ``seeds``); a sequence of temperatures
        (one per row, each >= 0; 0 = a greedy row) samples row b at temperature[b] in the
        same call (janus_whisper_decode_sample_rows_ex). ``enc_index`` (one int per
        decoder row): row b attends to enc[enc_index[b]] — the best_of hypotheses of a
        window share its encoder output, read once per pair of rows. ``pos_offset`` /
        ``steps`` (greedy): a staggered call — row b runs ``steps`` positions from
        pos_offset[b]; rows with an offset > 0 continue this context's previous call in the
        same row (pass the same batch size and their encoder output again), rows with 0
        start fresh (one contiguous range). ``state_slot``: the context's decoder state slot
        the call runs in (a sampled re-decode between two staggered calls takes another
        slot); ``logits_blocks`` / ``msplit_rows_n``: launch geometry (0 = measured
        defaults, janus_decode_options); ``persistent``: the persistent decoder segments
        (dec_persist.hip) where the shape allows; ``path_flags``: an alternative decoder path
        (DEC_PATH_*, parity tests)."""
        B = enc.shape[0] if enc_index is None else len(enc_index)
        if steps < 0:
            raise ValueError("steps must be >= 0")
        if steps and pos_offset is None:
            raise ValueError("steps applies to a staggered call (pos_offset) only")
        row_t = None
        if not np.isscalar(temperature):
            row_t = np.ascontiguousarray(np.asarray(temperature, np.float32))
            if row_t.shape != (B,) or not (row_t >= 0).all():
                raise ValueError("per-row temperatures: one value >= 0 per row")
            temperature = 1.0
        if temperature > 0:
            if seeds is None or len(seeds) != B:
                raise ValueError("sampling needs one uint32 seed per row")
            sd = np.ascontiguousarray(np.asarray(seeds, np.uint64) & 0xFFFFFFFF, dtype=np.uint32)
        opt, keep = self.decode_options(max_length, check_every, timestamps, xattn_splits, cu_count,
                                        state_slot, logits_blocks, msplit_rows_n, persistent,
                                        path_flags)
        rows = janus_decode_rows()
        rows.no_speech_token = tok.NO_SPEECH
        po = None
        if pos_offset is not None:
            po = np.ascontiguousarray(np.asarray(pos_offset, np.int32))
            if po.shape != (B,):
                raise ValueError("pos_offset needs one offset per row")
            rows.pos_offset = po.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            rows.steps = int(steps)
        ei = None
        if enc_index is not None:
            ei = np.ascontiguousarray(np.asarray(enc_index, np.int32))
            if ei.size and (ei.min() < 0 or ei.max() >= enc.shape[0]):
                raise ValueError("enc_index out of range")
            rows.enc_index = ei.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            rows.n_enc = int(enc.shape[0])
        plens = np.full(B, len(self.tokenizer.sot_sequence), np.int32)
        pr = None
        if prompts is not None:
            assert len(prompts) == B
            plens = np.array([len(p) for p in prompts], np.int32)
            stride = int(max(plens.max(), 1))
            pr = np.zeros((B, stride), np.int32)
            for b, p in enumerate(prompts):
                pr[b, :len(p)] = p
            rows.prompts = pr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            rows.prompt_lens = plens.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            rows.stride = stride
        tokens = torch.empty(B, max_length, dtype=torch.int32, device=self.device)
        ntok = torch.empty(B, dtype=torch.int32, device=self.device)
        slp = torch.empty(B, dtype=torch.float32, device=self.device)
        nsp = torch.empty(B, dtype=torch.float32, device=self.device)
        if row_t is not None:
            nat.call("janus_whisper_decode_sample_rows_ex", self._h, enc.data_ptr(), B,
                     ctypes.addressof(opt), ctypes.addressof(rows), row_t.ctypes.data,
                     sd.ctypes.data, tokens.data_ptr(), ntok.data_ptr(), slp.data_ptr(),
                     nsp.data_ptr(), nat.stream_ptr())
        elif temperature > 0:
            nat.call("janus_whisper_decode_sample_ex", self._h, enc.data_ptr(), B,
                     ctypes.addressof(opt), ctypes.addressof(rows), ctypes.c_float(temperature),
                     sd.ctypes.data, tokens.data_ptr(), ntok.data_ptr(), slp.data_ptr(),
                     nsp.data_ptr(), nat.stream_ptr())
        else:
            nat.call("janus_whisper_decode_greedy_ex", self._h, enc.data_ptr(), B, ctypes.addressof(opt),
                     ctypes.addressof(rows), tokens.data_ptr(), ntok.data_ptr(), slp.data_ptr(),
                     nsp.data_ptr(), nat.stream_ptr())
        del keep, pr, ei, po, row_t
        return DecodeOut(tokens, ntok, slp, nsp, plens)

    def decode_stand(self, batch: int, state_slot: int = 0):
        """Where each of the last decode call's ``batch`` row slots stands in decoder state
        slot ``state_slot`` (the largest pos_offset a staggered call may continue it from;
        janus_whisper_decode_stand_slot)."""
        out = np.zeros(batch, np.int32)
        nat.call("janus_whisper_decode_stand_slot", self._h, int(state_slot), out.ctypes.data,
                 int(batch))
        return [int(v) for v in out]

    def decode_check(self, state_slot: int = 0):
        """janus_whisper_decode_check: raise if the last non-polling call (check_every 0) of
        decoder state slot ``state_slot`` hit a persistent-segment barrier timeout (waits for
        that call's flag; nothing pending: returns at once). Call before using its outputs."""
        nat.call("janus_whisper_decode_check", self._h, int(state_slot))

    def decode_info(self):
        """(positions stepped, kernel launches issued) by the last decode call
        (janus_whisper_decode_info: captured graph nodes; measurement only)."""
        pos, lau = ctypes.c_int32(0), ctypes.c_int64(0)
        nat.call("janus_whisper_decode_info", self._h, ctypes.addressof(pos), ctypes.addressof(lau))
        return int(pos.value), int(lau.value)

    def texts(self, tokens: torch.Tensor, prompt_lens=None):
        """Host-side detokenisation of decoded rows (after each row's prompt)."""
        t = tokens.cpu().numpy()
        plen = len(self.tokenizer.sot_sequence)
        pl = prompt_lens if prompt_lens is not None else [plen] * len(t)
        return [self.tokenizer.transcript(row[int(p):]) for row, p in zip(t, pl)]


@dataclasses.dataclass
class DecodeOut:
    """Device tensors of one batched decode plus the host prompt lengths."""
    tokens: torch.Tensor          # int32 [B][max_length]: prompt, sampled tokens, -1
    n_tokens: torch.Tensor        # int32 [B]: sampled tokens incl. <|endoftext|>
    sum_logprob: torch.Tensor     # f32 [B]: sum of the chosen tokens' (filtered) log-probs
    no_speech_prob: torch.Tensor  # f32 [B]: raw P(<|nocaptions|>) at the first sampled step
    prompt_lens: np.ndarray       # int32 [B]

    def rows(self):
        """Per row: (sampled tokens without <|endoftext|>, avg_logprob, no_speech_prob),
        avg_logprob as faster-whisper derives it (sum / (len + 1), the +1 for eot)."""
        t, n = self.tokens.cpu().numpy(), self.n_tokens.cpu().numpy()
        lp, ns = self.sum_logprob.cpu().numpy(), self.no_speech_prob.cpu().numpy()
        out = []
        for b in range(len(n)):
            s = t[b][int(self.prompt_lens[b]):int(self.prompt_lens[b]) + int(n[b])]
            s = [int(x) for x in s if x != tok.EOT]
            out.append((s, float(lp[b]) / (len(s) + 1), float(ns[b])))
        return out
