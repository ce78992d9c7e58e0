"""Prosody extraction — drop-in for backend/services/prosody.py on MI355X.

``ProsodyExtractor`` keeps the reference's constructor, attributes
(``sample_rate``, ``hop_size``, ``pitch_detector``) and ``analyze_buffer`` contract
(prosody.py:11-104). RMS and per-hop aubio-YIN run in libjanus_hip.so
(``janus_prosody_analyze``); the detector's 4096-sample buffer persists on the GPU
across calls exactly like the one aubio.pitch object the reference builds once
(prosody.py:32) and calls per hop (:84). ``analyze_batch`` is the additive batched
form used by the pipeline and the bench (one independent stream per utterance).
"""
import threading

import numpy as np
import torch

from .. import _native as nat

YIN_BUF = 4096
DEFAULT_TOLERANCE = 0.8   # prosody.py:34
SILENCE_DB = -50.0        # aubio DEFAULT_PITCH_SILENCE (src/pitch/pitch.c)


def energy_tag(rms: float) -> str:
    """prosody.py:69-74 (NaN, from an empty buffer, falls through to 'Loud')."""
    if rms < 0.05:
        return 'Quiet'
    elif rms < 0.15:
        return 'Normal'
    return 'Loud'


def pitch_tag(mean_f0: float, n_voiced: int) -> str:
    """prosody.py:89-99."""
    if n_voiced > 0:
        if mean_f0 < 120:
            return 'Deep'
        elif mean_f0 < 200:
            return 'Normal'
        return 'High'
    return 'Normal'


def hop_offsets(lengths, hop: int) -> np.ndarray:
    nh = (np.asarray(lengths, np.int64) + hop - 1) // hop
    return np.concatenate([[0], np.cumsum(nh)]).astype(np.int64)


class ProsodyResult:
    """Device-resident outputs of one batched prosody launch."""

    def __init__(self, f0, rms, mean_f0, n_voiced, hop_off):
        self.f0, self.rms, self.mean_f0, self.n_voiced, self.hop_off = f0, rms, mean_f0, n_voiced, hop_off

    def tags(self):
        return self.tags_of(self.rms.cpu().numpy(), self.mean_f0.cpu().numpy(), self.n_voiced.cpu().numpy())

    @staticmethod
    def tags_of(rms, mf, nv):
        """The tags from host copies of (rms, mean_f0, n_voiced)."""
        return [{'energy': energy_tag(float(rms[b])), 'pitch': pitch_tag(float(mf[b]), int(nv[b]))}
                for b in range(len(rms))]


def prosody_launch(pcm: torch.Tensor, sample_offsets: torch.Tensor, lengths, sample_rate: int,
                   hop: int, tolerance: float = DEFAULT_TOLERANCE, silence_db: float = SILENCE_DB,
                   state_in: torch.Tensor = None, state_out: torch.Tensor = None,
                   max_blocks: int = 0) -> ProsodyResult:
    """Enqueue janus_prosody_analyze on the current stream; all tensors on the GPU."""
    B = len(lengths)
    dev = pcm.device
    assert pcm.dtype == torch.float32 and pcm.is_contiguous() and pcm.is_cuda
    ho_np = hop_offsets(lengths, hop)
    total = int(ho_np[-1])
    hop_off = torch.from_numpy(ho_np).pin_memory().to(dev, non_blocking=True)   # no host wait
    f0 = torch.empty(max(total, 1), dtype=torch.float32, device=dev)
    rms = torch.empty(max(B, 1), dtype=torch.float32, device=dev)
    mean_f0 = torch.empty(max(B, 1), dtype=torch.float32, device=dev)
    n_voiced = torch.empty(max(B, 1), dtype=torch.int32, device=dev)
    for t in (state_in, state_out):
        if t is not None:
            assert t.is_cuda and t.dtype == torch.float32 and t.numel() == B * YIN_BUF
    nat.call("janus_prosody_analyze_ex", pcm.data_ptr(), sample_offsets.data_ptr(), hop_off.data_ptr(),
             B, total, int(sample_rate), int(hop), float(tolerance), float(silence_db),
             state_in.data_ptr() if state_in is not None else None,
             state_out.data_ptr() if state_out is not None else None,
             f0.data_ptr(), rms.data_ptr(), mean_f0.data_ptr(), n_voiced.data_ptr(),
             int(max_blocks), nat.stream_ptr(dev))
    return ProsodyResult(f0[:total], rms[:B], mean_f0[:B], n_voiced[:B], ho_np)


class YinPitch:
    """Stand-in for the aubio.pitch('yin', 4096, hop, sr) object (prosody.py:32-34):
    owns the detector buffer on the GPU; calling it with one hop returns [f0]."""

    def __init__(self, buf_size: int, hop_size: int, sample_rate: int, device) -> None:
        if buf_size != YIN_BUF:
            raise ValueError("janus YIN is built for a 4096-sample buffer (prosody.py:32)")
        self.hop_size, self.sample_rate = hop_size, sample_rate
        self.tolerance = DEFAULT_TOLERANCE
        self.silence = SILENCE_DB
        self.unit = 'Hz'
        self.state = torch.zeros(YIN_BUF, dtype=torch.float32, device=device)
        self.lock = threading.Lock()

    def set_unit(self, unit: str) -> None:
        if unit not in ('Hz', 'hz', 'default', 'freq'):
            raise ValueError("janus YIN supports unit 'Hz' only")
        self.unit = unit

    def set_tolerance(self, tol: float) -> None:
        self.tolerance = float(tol)

    def set_silence(self, silence: float) -> None:
        self.silence = float(silence)

    def run(self, audio: np.ndarray) -> ProsodyResult:
        dev = self.state.device
        x = torch.from_numpy(np.ascontiguousarray(audio, np.float32)).to(dev)
        offs = torch.tensor([0, len(audio)], dtype=torch.int64, device=dev)
        with self.lock:
            new_state = torch.empty_like(self.state)
            res = prosody_launch(x, offs, [len(audio)], self.sample_rate, self.hop_size,
                                 self.tolerance, self.silence, self.state, new_state)
            self.state = new_state
            torch.cuda.current_stream(dev).synchronize()
        return res

    def __call__(self, chunk) -> np.ndarray:
        chunk = np.asarray(chunk, dtype=np.float32)
        if len(chunk) != self.hop_size:
            raise ValueError(f"input size {len(chunk)} != hop_size {self.hop_size}")
        return self.run(chunk).f0.cpu().numpy()


class ProsodyExtractor:
    def __init__(self, sample_rate: int = 48000, hop_size: int = 512) -> None:
        """Same contract as prosody.py:11-34."""
        self.device = nat.require_gpu()
        self.sample_rate = sample_rate
        self.hop_size = hop_size
        self.pitch_detector = YinPitch(YIN_BUF, hop_size, sample_rate, self.device)
        self.pitch_detector.set_unit('Hz')
        self.pitch_detector.set_tolerance(0.8)

    def analyze_buffer(self, audio_buffer: np.ndarray) -> dict[str, str]:
        """prosody.py:36-104: {'energy': Quiet|Normal|Loud, 'pitch': Deep|Normal|High}."""
        if isinstance(audio_buffer, list):
            audio_buffer = np.concatenate(audio_buffer)
        if not isinstance(audio_buffer, np.ndarray):
            audio_buffer = np.array(audio_buffer, dtype=np.float32)
        if audio_buffer.dtype != np.float32:
            audio_buffer = audio_buffer.astype(np.float32)
        res = self.pitch_detector.run(audio_buffer)
        return res.tags()[0]

    def analyze_batch(self, pcm: torch.Tensor, sample_offsets: torch.Tensor, lengths,
                      states_in: torch.Tensor = None,
                      states_out: torch.Tensor = None) -> ProsodyResult:
        """Batched extension: independent utterances packed back to back on the GPU."""
        return prosody_launch(pcm, sample_offsets, lengths, self.sample_rate, self.hop_size,
                              self.pitch_detector.tolerance, self.pitch_detector.silence,
                              states_in, states_out)
