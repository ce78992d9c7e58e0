"""Firefly-GAN vocoder host side: config, weights, prompt front end, GPU engine, WAV.

The reference's decode is a cloud call (synthesizer.py:191-203: Fish Audio
``tts.convert(text="(emotion) text", format="wav")``). Locally, the same prompt drives
a build-defined front end and the fish-speech Firefly-GAN generator
(HiFiGANGenerator: conv_pre k13; upsample rates 8,8,2,2,2 with kernels 16,16,4,4,4;
ParallelBlock of ResBlock1 with kernels 3,7,11 x dilations 1,3,5; SiLU; conv_post k13;
tanh; 44.1 kHz, hop 512):

  latent[f] = text_embed[prompt_byte[floor(f * n / F)]] + emotion_embed[emotion]

where ``emotion`` indexes the tag the reference puts in parentheses
(synthesizer.py:149-177). Without a checkpoint (``JANUS_VOCODER_DIR`` with
``model.safetensors``) the weights are seeded synthetic tensors of the real shapes.
"""
import ctypes
import dataclasses
import math
import os
import struct

import numpy as np
import torch

from . import _native as nat

SAMPLE_RATE = 44100
FRAMES_PER_BYTE = 6  # ~70 ms of audio per prompt byte for the drop-in path
EMOTIONS = ("relaxed", "excited", "joyful", "whispering", "shouting", "sad")


@dataclasses.dataclass(frozen=True)
class FireflyConfig:
    latent_dim: int = 512
    channels: int = 512
    up_rates: tuple = (8, 8, 2, 2, 2)
    rb_kernels: tuple = (3, 7, 11)
    rb_dilations: tuple = (1, 3, 5)
    pre_kernel: int = 13
    post_kernel: int = 13
    n_emotions: int = 16
    n_voices: int = 16

    @property
    def hop(self):
        return int(np.prod(self.up_rates))


class janus_vocoder_config(ctypes.Structure):
    _fields_ = [("latent_dim", ctypes.c_int), ("channels", ctypes.c_int), ("n_ups", ctypes.c_int),
                ("up_rates", ctypes.c_int * 8), ("n_kernels", ctypes.c_int),
                ("rb_kernels", ctypes.c_int * 4), ("n_dilations", ctypes.c_int),
                ("rb_dilations", ctypes.c_int * 4), ("pre_kernel", ctypes.c_int),
                ("post_kernel", ctypes.c_int), ("n_emotions", ctypes.c_int)]


def _fnv1a(s: str) -> int:
    h = 0x811C9DC5
    for b in s.encode("utf-8"):
        h = ((h ^ b) * 0x01000193) & 0xFFFFFFFF
    return h


def emotion_id(tag: str, n_emotions: int = 16) -> int:
    """Known prompt tags map to fixed rows; any other override string (synthesizer.py:150-151)
    to a stable FNV-1a bucket of the remaining rows."""
    t = str(tag).lower()
    if t in EMOTIONS:
        return EMOTIONS.index(t)
    return len(EMOTIONS) + _fnv1a(t) % (n_emotions - len(EMOTIONS))


# the reference's stock voice when no recording is loaded (synthesizer.py:189)
DEFAULT_REFERENCE_ID = "5196af35f6ff4a0dbf541793fc9f2157"


def voice_id(reference_id: str, n_voices: int = 16) -> int:
    """Row of frontend.voice_embed for a Fish voice id (FNV-1a bucket)."""
    return _fnv1a(str(reference_id)) % n_voices


def split_prompt(text: str):
    """Fish-style prompt "(tag) text" -> (tag, text); no leading tag -> (None, text).
    The reference builds exactly this form (synthesizer.py:152, :177, :231)."""
    if text.startswith("(") and ") " in text:
        i = text.index(") ")
        return text[1:i], text[i + 2:]
    return None, text


def synthetic_weights(cfg: FireflyConfig, seed: int = 0) -> dict:
    g = torch.Generator().manual_seed(seed)
    W = {}

    def rn(name, *shape, std):
        W[name] = (torch.randn(*shape, generator=g) * std).numpy().astype(np.float32)

    rn("frontend.text_embed", 256, cfg.latent_dim, std=1.0)
    rn("frontend.emotion_embed", cfg.n_emotions, cfg.latent_dim, std=0.5)
    C = cfg.channels
    rn("conv_pre.weight", C, cfg.latent_dim, cfg.pre_kernel, std=1.0 / math.sqrt(cfg.latent_dim * cfg.pre_kernel))
    rn("conv_pre.bias", C, std=0.02)
    for i, u in enumerate(cfg.up_rates):
        rn(f"ups.{i}.weight", C, C // 2, 2 * u, std=2.0 / math.sqrt(C * 2))
        rn(f"ups.{i}.bias", C // 2, std=0.02)
        C //= 2
        for j, k in enumerate(cfg.rb_kernels):
            for m, d in enumerate(cfg.rb_dilations):
                p = f"resblocks.{i}.blocks.{j}"
                rn(f"{p}.convs1.{m}.weight", C, C, k, std=1.0 / math.sqrt(C * k))
                rn(f"{p}.convs1.{m}.bias", C, std=0.02)
                rn(f"{p}.convs2.{m}.weight", C, C, k, std=0.5 / math.sqrt(C * k))
                rn(f"{p}.convs2.{m}.bias", C, std=0.02)
    rn("conv_post.weight", 1, C, cfg.post_kernel, std=0.35 / math.sqrt(C * cfg.post_kernel))
    rn("conv_post.bias", 1, std=0.02)
    # voice conditioning (appended last: the tensors above keep their seeded values)
    rn("frontend.speaker_proj", cfg.latent_dim, 80, std=0.5 / math.sqrt(80))
    rn("frontend.speaker_bias", cfg.latent_dim, std=0.02)
    rn("frontend.voice_embed", cfg.n_voices, cfg.latent_dim, std=0.5)
    return W


def load_weights(cfg: FireflyConfig, seed: int = 0) -> dict:
    path = os.environ.get("JANUS_VOCODER_DIR")
    if path and os.path.exists(os.path.join(path, "model.safetensors")):
        from safetensors.numpy import load_file
        return {k: v.astype(np.float32) for k, v in load_file(os.path.join(path, "model.safetensors")).items()}
    return synthetic_weights(cfg, seed)


def wav_bytes(pcm: np.ndarray, sample_rate: int = SAMPLE_RATE) -> bytes:
    """44-byte RIFF/WAVE header + mono int16 PCM (the layout of
    backend/tests/test_e2e_local.py:79-101)."""
    pcm = np.ascontiguousarray(pcm, dtype="<i2")
    data_size = pcm.size * 2
    header = struct.pack('<4sI4s4sIHHIIHH4sI', b'RIFF', 36 + data_size, b'WAVE', b'fmt ', 16, 1, 1,
                         sample_rate, sample_rate * 2, 2, 16, b'data', data_size)
    return header + pcm.tobytes()


class VocoderEngine:
    def __init__(self, cfg: FireflyConfig = FireflyConfig(), weights: dict = None, seed: int = 0):
        self.device = nat.require_gpu()
        self.cfg = cfg
        c = janus_vocoder_config()
        c.latent_dim, c.channels = cfg.latent_dim, cfg.channels
        c.n_ups = len(cfg.up_rates)
        for i, u in enumerate(cfg.up_rates):
            c.up_rates[i] = u
        c.n_kernels = len(cfg.rb_kernels)
        for i, k in enumerate(cfg.rb_kernels):
            c.rb_kernels[i] = k
        c.n_dilations = len(cfg.rb_dilations)
        for i, d in enumerate(cfg.rb_dilations):
            c.rb_dilations[i] = d
        c.pre_kernel, c.post_kernel, c.n_emotions = cfg.pre_kernel, cfg.post_kernel, cfg.n_emotions
        h = ctypes.c_void_p()
        nat.call("janus_vocoder_create", ctypes.addressof(c), ctypes.addressof(h))
        self._h = h
        weights = dict(weights if weights is not None else load_weights(cfg, seed))
        # host copy of what was uploaded: a second context with the same weights (the
        # staggered step's decoder-side renders) is built from it, never re-derived
        self.weights = weights
        from .whisper import mel_constants  # the speaker path's log-mel front end
        weights["mel.basis"], weights["mel.filters"] = mel_constants()
        for name, arr in weights.items():
            a = np.ascontiguousarray(arr, dtype=np.float32)
            nat.call("janus_vocoder_set_tensor", self._h, name.encode(), a.ctypes.data, a.size)
        ve = weights.get("frontend.voice_embed")
        self._voices = (torch.from_numpy(np.ascontiguousarray(ve, np.float32)).to(self.device)
                        if ve is not None else None)
        self.has_speaker = "frontend.speaker_proj" in weights

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                nat.lib().janus_vocoder_destroy(h)
            except Exception:
                pass

    def frontend(self, prompts, emotions, frames: int, speaker: torch.Tensor = None) -> torch.Tensor:
        """prompts: list of bytes; emotions: list of int ids; speaker: optional f32 device
        tensor [B][latent] (voice term per row) -> latents fp16 [B][F][latent]."""
        B = len(prompts)
        offs = np.concatenate([[0], np.cumsum([len(p) for p in prompts])]).astype(np.int64)
        allb = np.frombuffer(b"".join(prompts) + b"\0", np.uint8).copy()
        # pinned, non-blocking uploads: a pageable copy would hold the host until the stream
        # reaches it (the serving step issues this behind its encoders)
        up = lambda a: torch.from_numpy(a).pin_memory().to(self.device, non_blocking=True)  # noqa: E731
        d_bytes = up(allb)
        d_offs = up(offs)
        d_emo = up(np.asarray(list(emotions), np.int32))
        lat = torch.empty(B, frames, self.cfg.latent_dim, dtype=torch.float16, device=self.device)
        spk_ptr = None
        if speaker is not None:
            assert speaker.shape == (B, self.cfg.latent_dim) and speaker.dtype == torch.float32
            speaker = speaker.contiguous()
            spk_ptr = speaker.data_ptr()
        nat.call("janus_vocoder_frontend_ex", self._h, d_bytes.data_ptr(), d_offs.data_ptr(),
                 d_emo.data_ptr(), spk_ptr, B, frames, lat.data_ptr(), nat.stream_ptr())
        return lat

    def speaker_embedding(self, clips16k) -> torch.Tensor:
        """Voice vectors [B][latent] f32 (device) of reference recordings given as 16 kHz
        f32 arrays (the first 30 s of each is used)."""
        if not self.has_speaker:
            raise RuntimeError("vocoder weights have no frontend.speaker_proj")
        clips = [np.ascontiguousarray(c, np.float32)[:480000] for c in clips16k]
        B = len(clips)
        offs = torch.from_numpy(np.concatenate([[0], np.cumsum([len(c) for c in clips])]).astype(np.int64)).to(self.device)
        pcm = torch.from_numpy(np.concatenate(clips + [np.zeros(1, np.float32)])).to(self.device)
        out = torch.empty(B, self.cfg.latent_dim, dtype=torch.float32, device=self.device)
        nat.call("janus_vocoder_speaker", self._h, pcm.data_ptr(), offs.data_ptr(), B,
                 out.data_ptr(), nat.stream_ptr())
        return out

    def voice(self, reference_id: str) -> torch.Tensor:
        """Voice vector [latent] of a stock voice id (frontend.voice_embed row)."""
        if self._voices is None:
            raise RuntimeError("vocoder weights have no frontend.voice_embed")
        return self._voices[voice_id(reference_id, self._voices.shape[0])]

    def forward(self, lat: torch.Tensor, want_pcm: bool = True, want_pre_tanh: bool = False):
        """-> (wav f32, pcm int16 | None) or, with want_pre_tanh, (wav, pcm, conv_post out)."""
        B, Fr, _ = lat.shape
        T = Fr * self.cfg.hop
        wav = torch.empty(B, T, dtype=torch.float32, device=self.device)
        pcm = torch.empty(B, T, dtype=torch.int16, device=self.device) if want_pcm else None
        pre = torch.empty(B, T, dtype=torch.float32, device=self.device) if want_pre_tanh else None
        nat.call("janus_vocoder_forward_ex", self._h, lat.data_ptr(), B, Fr, wav.data_ptr(),
                 pcm.data_ptr() if pcm is not None else None,
                 pre.data_ptr() if pre is not None else None, nat.stream_ptr())
        return (wav, pcm, pre) if want_pre_tanh else (wav, pcm)

    def set_timing(self, on: bool) -> None:
        nat.call("janus_vocoder_set_timing", self._h, int(on))

    def family_stats(self, reset: bool = True):
        """{family: dict(flops, bytes, ms, launches)} of the timed launches; family = the
        fused unit's channel width, 0 = conv kernel (conv_pre, upsamplers)."""
        cap = 8
        fam = (ctypes.c_int * cap)()
        fl, by, ms = (ctypes.c_double * cap)(), (ctypes.c_double * cap)(), (ctypes.c_double * cap)()
        la = (ctypes.c_int64 * cap)()
        n = ctypes.c_int()
        nat.call("janus_vocoder_family_stats", self._h, cap, fam, fl, by, ms, la, ctypes.addressof(n),
                 int(reset))
        return {fam[i]: dict(flops=fl[i], bytes=by[i], ms=ms[i], launches=la[i]) for i in range(n.value)}

    def conv_stats(self, reset: bool = True):
        fl, ms, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        nat.call("janus_vocoder_conv_stats", self._h, ctypes.addressof(fl), ctypes.addressof(ms),
                 ctypes.addressof(n), int(reset))
        return fl.value, ms.value, n.value
