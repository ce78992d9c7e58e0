"""Voice activity detection — drop-in for backend/services/vad.py on MI355X.

Same constructor, ``is_speech`` and ``reset`` as the reference (vad.py:10-88), which runs
silero-vad (fetched by torch.hub — unreachable offline) on ``chunk[::3]`` at 16 kHz.

* With local silero weights (``JANUS_VAD_DIR/model.safetensors`` under silero's state-dict
  names, or ``weights=``) the neural gate runs on the GPU (csrc/vad.hip, janus_vad_run):
  silero-vad v5's 16 kHz graph with its per-object state (64-sample context + LSTM h, c)
  carried across calls as the reference's model object carries it.
* Without weights: the documented energy stand-in (janus_vad_energy, same x[::3] view
  and threshold contract): P(speech) = sigmoid((dB - center) / width).

``MultiStreamGate`` runs the chosen gate for S channels at once (one state per channel).
"""
import ctypes
import math
import os

import numpy as np
import torch

from .. import _native as nat

# energy stand-in for silero (vad.py:40-77): P(speech) = sigmoid((dB - center) / width)
VAD_CENTER_DB = -45.0
VAD_WIDTH_DB = 3.0
CTX, HID = 64, 128


def stft_basis(n_fft: int = 256) -> np.ndarray:
    """silero's STFT forward basis: [real rows 0..n/2 | imaginary rows] of the DFT, scaled
    by a periodic Hann window: [258][256]."""
    fb = np.fft.fft(np.eye(n_fft))
    cut = n_fft // 2 + 1
    fb = np.vstack([np.real(fb[:cut]), np.imag(fb[:cut])])
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft)
    return (fb * win[None, :]).astype(np.float32)


def synthetic_weights(seed: int = 0) -> dict:
    """Seeded silero-vad v5 (16 kHz) shaped weights under the published names."""
    g = torch.Generator().manual_seed(seed)
    W = {"_model.stft.forward_basis_buffer": stft_basis()[:, None, :]}

    def rn(name, *shape, std):
        W[name] = (torch.randn(*shape, generator=g) * std).numpy().astype(np.float32)

    for i, (ci, co) in enumerate([(129, 128), (128, 64), (64, 64), (64, 128)]):
        rn(f"_model.encoder.{i}.reparam_conv.weight", co, ci, 3, std=1.0 / math.sqrt(ci * 3))
        rn(f"_model.encoder.{i}.reparam_conv.bias", co, std=0.02)
    for n in ("weight_ih", "weight_hh"):
        rn(f"_model.decoder.rnn.{n}", 4 * HID, HID, std=1.0 / math.sqrt(HID))
    for n in ("bias_ih", "bias_hh"):
        rn(f"_model.decoder.rnn.{n}", 4 * HID, std=0.05)
    rn("_model.decoder.decoder.2.weight", 1, HID, 1, std=1.0 / math.sqrt(HID))
    rn("_model.decoder.decoder.2.bias", 1, std=0.1)
    return W


def load_weights():
    """Silero weights from JANUS_VAD_DIR/model.safetensors (16 kHz branch names), or None."""
    path = os.environ.get("JANUS_VAD_DIR")
    if path and os.path.exists(os.path.join(path, "model.safetensors")):
        from safetensors.numpy import load_file
        raw = load_file(os.path.join(path, "model.safetensors"))
        return {k: v.astype(np.float32) for k, v in raw.items()}
    return None


class SileroGate:
    """One janus_vad context (weights on the device); state buffers are the caller's."""

    def __init__(self, weights: dict):
        self.device = nat.require_gpu()
        h = ctypes.c_void_p()
        nat.call("janus_vad_create", ctypes.addressof(h))
        self._h = h
        for name, arr in weights.items():
            a = np.ascontiguousarray(arr, dtype=np.float32)
            nat.call("janus_vad_set_tensor", self._h, name.encode(), a.ctypes.data, a.size)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                nat.lib().janus_vad_destroy(h)
            except Exception:
                pass

    def new_state(self, n_streams: int):
        return (torch.zeros(n_streams, CTX, dtype=torch.float32, device=self.device),
                torch.zeros(n_streams, 2, HID, dtype=torch.float32, device=self.device))

    def run(self, pcm: torch.Tensor, state, decim: int) -> torch.Tensor:
        """pcm [S][n][L] f32 (device) -> probabilities [S][n]; state updated in place."""
        assert pcm.is_cuda and pcm.dtype == torch.float32 and pcm.dim() == 3
        pcm = pcm.contiguous()
        S, n, L = pcm.shape
        ctx, hc = state
        prob = torch.empty(max(S * n, 1), dtype=torch.float32, device=pcm.device)
        nat.call("janus_vad_run", self._h, pcm.data_ptr(), S, n, L, decim, ctx.data_ptr(),
                 hc.data_ptr(), prob.data_ptr(), nat.stream_ptr(pcm.device))
        return prob[:S * n].reshape(S, n)


def _energy_prob(chunks: torch.Tensor, decim: int) -> torch.Tensor:
    assert chunks.is_cuda and chunks.dtype == torch.float32 and chunks.is_contiguous()
    n, L = chunks.shape
    prob = torch.empty(max(n, 1), dtype=torch.float32, device=chunks.device)
    nat.call("janus_vad_energy", chunks.data_ptr(), n, L, decim, VAD_CENTER_DB, VAD_WIDTH_DB,
             prob.data_ptr(), nat.stream_ptr(chunks.device))
    return prob[:n]


class VoiceActivityDetector:
    """vad.py:10-88: same constructor / is_speech / reset, plus the batched GPU form.
    ``weights``: silero state dict (default: JANUS_VAD_DIR, else the energy stand-in)."""

    def __init__(self, threshold: float = 0.5, sample_rate: int = 48000, weights: dict = None) -> None:
        self.device = nat.require_gpu()
        self.threshold = threshold
        self.sample_rate = sample_rate
        self.decim = 3 if sample_rate in (48000, 44100) else 1  # vad.py:52-60
        w = weights if weights is not None else load_weights()
        self.model = SileroGate(w) if w is not None else None
        self._state = self.model.new_state(1) if self.model is not None else None

    def probabilities(self, chunks: torch.Tensor) -> torch.Tensor:
        """chunks: [N][L] f32 on the GPU, consecutive chunks of ONE stream -> [N] speech
        probabilities (the neural gate advances this detector's state through them)."""
        if self.model is None:
            return _energy_prob(chunks, self.decim)
        return self.model.run(chunks.reshape(1, *chunks.shape), self._state, self.decim)[0]

    def is_speech_batch(self, chunks: torch.Tensor) -> np.ndarray:
        return (self.probabilities(chunks) > self.threshold).cpu().numpy()

    def is_speech(self, audio_chunk) -> bool:
        """vad.py:40-77: speech_prob(chunk[::3] @ 16 kHz) > threshold."""
        x = torch.as_tensor(np.ascontiguousarray(audio_chunk, np.float32)).to(self.device)
        return bool(self.is_speech_batch(x.reshape(1, -1))[0])

    def reset(self) -> None:
        """A no-op, as in the reference (vad.py:79-88): the model state is kept."""


class MultiStreamGate:
    """The gate for S capture channels at once, one detector state per channel."""

    def __init__(self, n_streams: int, threshold: float = 0.5, sample_rate: int = 48000,
                 weights: dict = None):
        self.det = VoiceActivityDetector(threshold, sample_rate, weights)
        self.S = n_streams
        self.state = self.det.model.new_state(n_streams) if self.det.model is not None else None

    @property
    def neural(self) -> bool:
        return self.det.model is not None

    def probabilities(self, chunks: torch.Tensor) -> torch.Tensor:
        """chunks [S][n][L] (device) -> [S][n]."""
        S, n, L = chunks.shape
        if self.det.model is None:
            return _energy_prob(chunks.reshape(S * n, L).contiguous(), self.det.decim).reshape(S, n)
        return self.det.model.run(chunks, self.state, self.det.decim)

    def is_speech(self, chunks: torch.Tensor) -> np.ndarray:
        return (self.probabilities(chunks) > self.det.threshold).cpu().numpy()
