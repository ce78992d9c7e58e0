"""Speech-to-text — drop-in for backend/services/transcriber.py on MI355X.

``Transcriber`` keeps the reference's constructor and methods (transcriber.py:11-91) and
even its body: it builds ``WhisperModel(model_size, device=..., compute_type=...)`` and
iterates ``model.transcribe(audio[::3], beam_size=1, language='en')`` segments. Here
``WhisperModel`` is the GPU engine (log-mel, encoder and greedy decoder in
libjanus_hip.so) behind faster-whisper's call shape (``transcribe`` returns
``(segments, info)``; segments carry ``.text``), so module-level patching of
``WhisperModel`` in tests works exactly as in the reference suite
(backend/tests/test_input_processing.py:73-90).

Scope: greedy temperature-0 decoding of 30 s windows with the Whisper logit rules;
faster-whisper's temperature fallback (compression-ratio / log-prob gates with sampling
at T > 0), no-speech skipping and timestamp-seek re-decoding are not reproduced; audio
longer than 30 s is cut into consecutive 30 s windows.
"""
import dataclasses

import numpy as np
import torch

from .. import _native as nat
from ..common import wavio
from ..whisper import CONFIGS, WhisperEngine

WINDOW_16K = 480000


@dataclasses.dataclass
class Segment:
    id: int
    start: float
    end: float
    text: str
    tokens: list
    avg_logprob: float


@dataclasses.dataclass
class TranscriptionInfo:
    language: str
    language_probability: float
    duration: float


read_wav_16k = wavio.read_wav_16k  # 16-bit PCM WAV -> f32 @ 16 kHz

# faster-whisper's device / compute_type vocabulary (WhisperModel(model_size, device=...,
# compute_type=...)); every value names the SAME GPU engine here (see WhisperModel)
DEVICES = ("cpu", "cuda", "auto")
COMPUTE_TYPES = ("default", "auto", "int8", "int8_float32", "int8_float16", "int8_bfloat16",
                 "int16", "float16", "bfloat16", "float32")


class WhisperModel:
    """faster-whisper-shaped front of the GPU Whisper engine.

    Accepts faster-whisper's constructor arguments, including the reference's
    ``device='cpu', compute_type='int8'`` (transcriber.py:23-27), and maps every
    combination onto the one engine this build has: the gfx950 HIP kernels on the
    current device, with fp16 weights on MFMA and fp32 accumulation (the decoder's
    activations carried at fp32 precision as split-fp16 operands). ``device`` and
    ``compute_type`` are recorded (``requested_device`` / ``requested_compute_type``)
    but select nothing: there is no CPU path (the product fails loudly without a GPU)."""

    def __init__(self, model_size: str, device: str = "auto", compute_type: str = "default",
                 **_ignored):
        if model_size not in CONFIGS:
            raise ValueError(f"unknown model size {model_size!r}; one of {sorted(CONFIGS)}")
        if device not in DEVICES:
            raise ValueError(f"unsupported device {device!r}; one of {DEVICES}")
        if compute_type not in COMPUTE_TYPES:
            raise ValueError(f"unsupported compute_type {compute_type!r}")
        self.model_size = model_size
        self.requested_device, self.requested_compute_type = device, compute_type
        self.engine = WhisperEngine(CONFIGS[model_size])

    def transcribe(self, audio, beam_size: int = 1, language: str = "en", **_ignored):
        if beam_size != 1:
            raise NotImplementedError("janus_amd decodes greedily (beam_size=1, transcriber.py:55)")
        if isinstance(audio, str):
            audio = read_wav_16k(audio)
        audio = np.ascontiguousarray(audio, dtype=np.float32)
        eng = self.engine
        dev = eng.device
        windows = [audio[i:i + WINDOW_16K] for i in range(0, max(len(audio), 1), WINDOW_16K)]
        lengths = [len(w) for w in windows]
        offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
        pcm = torch.from_numpy(np.concatenate(windows + [np.zeros(1, np.float32)])).to(dev)
        mel = eng.logmel(pcm, offs, len(windows), 1)
        enc = eng.encode(mel)
        tokens, ntok, slp = eng.decode(enc)
        toks = tokens.cpu().numpy()
        nt = ntok.cpu().numpy()
        lp = slp.cpu().numpy()
        tk = eng.tokenizer
        plen = len(tk.sot_sequence)
        segs = []
        for w in range(len(windows)):
            base = w * 30.0
            avg = float(lp[w] / max(int(nt[w]), 1))
            for (s, e, text) in tk.segments(toks[w][plen:]):
                segs.append(Segment(len(segs), base + s, base + e, text,
                                    [int(t) for t in toks[w][plen:plen + int(nt[w])]], avg))
        info = TranscriptionInfo(language, 1.0, len(audio) / 16000.0)
        return iter(segs), info


class Transcriber:
    def __init__(self, model_size: str = 'base.en') -> None:
        """transcriber.py:11-27, the same call (WhisperModel maps it onto the GPU engine)."""
        self.model = WhisperModel(
            model_size,
            device='cpu',
            compute_type='int8'
        )

    def transcribe_buffer(self, audio_buffer: np.ndarray) -> str:
        """transcriber.py:29-64."""
        if isinstance(audio_buffer, list):
            audio_buffer = np.concatenate(audio_buffer)
        if not isinstance(audio_buffer, np.ndarray):
            audio_buffer = np.array(audio_buffer, dtype=np.float32)
        if audio_buffer.dtype != np.float32:
            audio_buffer = audio_buffer.astype(np.float32)
        audio_16k = audio_buffer[::3]
        segments, info = self.model.transcribe(audio_16k, beam_size=1, language='en')
        text_parts = []
        for segment in segments:
            text_parts.append(segment.text.strip())
        full_text = ' '.join(text_parts).strip()
        return full_text

    def transcribe_file(self, file_path: str) -> str:
        """transcriber.py:66-91 (16-bit PCM WAV input)."""
        segments, info = self.model.transcribe(file_path, beam_size=1, language='en')
        text_parts = []
        for segment in segments:
            text_parts.append(segment.text.strip())
        full_text = ' '.join(text_parts).strip()
        return full_text

    def transcribe_batch(self, buffers) -> list:
        """Batched extension: 48 kHz buffers (<= 30 s each) -> transcripts, one GPU pass."""
        eng = self.model.engine
        dev = eng.device
        bufs = [np.ascontiguousarray(b, dtype=np.float32)[:3 * WINDOW_16K] for b in buffers]
        lengths = [len(b) for b in bufs]
        offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=dev)
        pcm = torch.from_numpy(np.concatenate(bufs + [np.zeros(1, np.float32)])).to(dev)
        tokens, _, _ = eng.decode(eng.encode(eng.logmel(pcm, offs, len(bufs), 3)))
        return eng.texts(tokens)


__all__ = ["Transcriber", "WhisperModel", "Segment", "TranscriptionInfo", "read_wav_16k", "nat"]
