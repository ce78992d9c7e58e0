"""Speech-to-text — drop-in for backend/services/transcriber.py on MI355X.

``Transcriber`` keeps the reference's constructor and methods (transcriber.py:11-91) and
even its body: it builds ``WhisperModel(model_size, device='cpu', compute_type='int8')``
and iterates ``model.transcribe(audio[::3], beam_size=1, language='en')`` segments. Here
``WhisperModel`` is the GPU engine (log-mel, encoder and greedy decoder in
libjanus_hip.so) behind faster-whisper's call shape (``transcribe`` returns
``(segments, info)``; segments carry ``.text`` and the decode statistics), so
module-level patching of ``WhisperModel`` in tests works exactly as in the reference
suite (backend/tests/test_input_processing.py:73-90).

``transcribe`` restates faster-whisper's ``generate_segments`` loop for the reference's
call (beam_size=1, language='en', every other option at its default):

* windows of 3000 log-mel frames at a moving ``seek``; the next seek is the end of the
  window when the tokens end in a single timestamp or hold none, else the last
  consecutive-timestamp pair (the trailing partial segment is re-decoded from there);
* ``condition_on_previous_text``: each window's prompt is ``<|startofprev|>`` + the
  last <= 223 tokens of the segments emitted so far + ``<|startoftranscript|>``;
* the gates, computed per window: ``avg_logprob`` = sum of chosen-token log-probs /
  (tokens + 1), ``compression_ratio`` = len(text) / len(zlib(text)),
  ``no_speech_prob`` = raw P(<|nocaptions|>) at the first step (on the GPU);
  no-speech skip when no_speech_prob > 0.6 and avg_logprob <= -1;
* segments whose start equals their end or whose text is blank are dropped.

Deliberate deviations: the temperature FALLBACK is not run — a window
whose gates fail (compression ratio > 2.4 or avg_logprob < -1, outside the no-speech
case) is flagged (``Segment.needs_fallback``, ``WhisperModel.stats``) and its T = 0
decode kept, because the T > 0 re-decodes are random samples no offline oracle can pin;
a window that would not advance the seek (a leading <|0.00|><|0.00|>) advances by the
window size, so the loop always terminates.

Features are faster-whisper's: one log-mel of the whole clip (normalised with the maximum
over all its frames), from which each window takes the content frames
[seek, seek + min(3000, content - seek)) and is padded with zeros to 3000 frames
(``features[:, seek:seek + segment_size]`` + ``pad_or_trim``).
"""
import dataclasses
import zlib

import numpy as np
import torch

from .. import _native as nat
from ..common import wavio
from ..tokenizer import SOT_PREV
from ..whisper import CONFIGS, WhisperEngine

WINDOW_16K = 480000
N_FRAMES = 3000          # log-mel frames per window (hop 160 @ 16 kHz)
HOP = 160
TIME_PRECISION = 0.02    # seconds per timestamp step
INPUT_STRIDE = 2         # mel frames per timestamp step
COMPRESSION_RATIO_THRESHOLD = 2.4
LOG_PROB_THRESHOLD = -1.0
NO_SPEECH_THRESHOLD = 0.6


@dataclasses.dataclass
class Segment:
    id: int
    seek: int
    start: float
    end: float
    text: str
    tokens: list
    temperature: float
    avg_logprob: float
    compression_ratio: float
    no_speech_prob: float
    needs_fallback: bool = False


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


def compression_ratio(text: str) -> float:
    """faster-whisper get_compression_ratio."""
    b = text.encode("utf-8")
    return len(b) / len(zlib.compress(b))


def gates(text: str, avg_logprob: float, no_speech_prob: float):
    """(needs_fallback, no_speech_skip) for one T = 0 window, faster-whisper's rules."""
    needs = compression_ratio(text) > COMPRESSION_RATIO_THRESHOLD or avg_logprob < LOG_PROB_THRESHOLD
    if no_speech_prob > NO_SPEECH_THRESHOLD and avg_logprob < LOG_PROB_THRESHOLD:
        needs = False                      # silence: no fallback
    skip = no_speech_prob > NO_SPEECH_THRESHOLD and not avg_logprob > LOG_PROB_THRESHOLD
    return needs, skip


def split_window(tk, tokens, seek, segment_size):
    """One window's tokens -> ([(start_s, end_s, tokens)], next seek) as faster-whisper's
    generate_segments slices them (timestamps included in the token lists)."""
    tb = tk.timestamp_begin
    time_offset = seek * HOP / 16000.0
    single_ending = len(tokens) >= 2 and tokens[-2] < tb <= tokens[-1]
    consecutive = [i for i in range(1, len(tokens)) if tokens[i] >= tb and tokens[i - 1] >= tb]
    segs = []
    if consecutive:
        slices = list(consecutive)
        if single_ending:
            slices.append(len(tokens))
        last = 0
        for cur in slices:
            part = tokens[last:cur]
            segs.append((time_offset + (part[0] - tb) * TIME_PRECISION,
                         time_offset + (part[-1] - tb) * TIME_PRECISION, part))
            last = cur
        if single_ending:
            nseek = seek + segment_size
        else:
            nseek = seek + (tokens[last - 1] - tb) * INPUT_STRIDE
    else:
        duration = segment_size * HOP / 16000.0
        stamps = [t for t in tokens if t >= tb]
        if stamps and stamps[-1] != tb:
            duration = (stamps[-1] - tb) * TIME_PRECISION
        segs.append((time_offset, time_offset + duration, tokens))
        nseek = seek + segment_size
    if nseek <= seek:          # no progress (e.g. <|0.00|><|0.00|>): move on a window
        nseek = seek + segment_size
    return segs, nseek


class _Stream:
    """generate_segments state of one utterance."""

    def __init__(self, audio16k):
        self.audio = audio16k
        self.content_frames = len(audio16k) // HOP
        self.seek = 0
        self.all_tokens = []
        self.prompt_reset_since = 0
        self.segments = []
        self.windows = self.fallbacks = self.skips = 0

    @property
    def active(self):
        return self.seek < self.content_frames

    def window_size(self):
        return min(N_FRAMES, self.content_frames - self.seek)

    def prompt(self, tk, max_length=448):
        prev = self.all_tokens[self.prompt_reset_since:]
        p = ([SOT_PREV] + prev[-(max_length // 2 - 1):]) if prev else []   # 223 at 448
        return p + list(tk.sot_sequence)


def generate_segments(engine: WhisperEngine, audios, max_batch: int = 64, max_length: int = 448):
    """faster-whisper's seek loop for several 16 kHz utterances at once: every round
    decodes the current window of each unfinished utterance as one GPU batch (per-row
    prompts). Returns one _Stream (segments + gate counters) per utterance."""
    tk = engine.tokenizer
    dev = engine.device
    streams = [_Stream(np.asarray(a, np.float32)) for a in audios]
    # the whole clip's features, once per utterance (faster-whisper's FeatureExtractor call)
    feats = []
    for st in streams:
        if st.content_frames <= 0:
            feats.append(None)
            continue
        pcm = torch.from_numpy(np.concatenate([st.audio, np.zeros(1, np.float32)])).to(dev)
        offs = torch.tensor([0, len(st.audio)], dtype=torch.int64, device=dev)
        feats.append(engine.logmel_frames(pcm, offs, 1, 1, st.content_frames)[0])
    while True:
        act = [i for i, s in enumerate(streams) if s.active]
        if not act:
            break
        for c0 in range(0, len(act), max_batch):
            idx = act[c0:c0 + max_batch]
            grp = [streams[i] for i in idx]
            sizes = [s.window_size() for s in grp]
            mel = torch.zeros(len(grp), N_FRAMES, 80, dtype=torch.float16, device=dev)
            for j, (i, s, size) in enumerate(zip(idx, grp, sizes)):
                mel[j, :size] = feats[i][s.seek:s.seek + size]      # pad_or_trim: zeros after
            enc = engine.encode(mel)
            out = engine.decode_ex(enc, prompts=[s.prompt(tk, max_length) for s in grp], max_length=max_length)
            wins = [(size, None) for size in sizes]
            for s, (size, _), (toks, avg_lp, nsp) in zip(grp, wins, out.rows()):
                s.windows += 1
                text = tk.decode(toks).strip()
                cr = compression_ratio(text)
                needs, skip = gates(text, avg_lp, nsp)
                s.fallbacks += int(needs)
                if skip:
                    s.skips += 1
                    s.seek += size
                    continue
                segs, nseek = split_window(tk, toks, s.seek, size)
                for (st, en, part) in segs:
                    txt = tk.decode(part)
                    if st == en or not txt.strip():
                        continue
                    s.all_tokens.extend(part)
                    s.segments.append(Segment(len(s.segments), s.seek, st, en, txt, part, 0.0,
                                              avg_lp, cr, nsp, needs))
                s.seek = nseek
                # condition_on_previous_text at temperature 0 <= prompt_reset_on_temperature:
                # the prompt is never reset
    return streams


class WhisperModel:
    """faster-whisper-shaped front of the GPU Whisper engine.

    Accepts faster-whisper's constructor arguments, including the reference's
    ``device='cpu', compute_type='int8'`` (transcriber.py:23-27), and maps every
    combination onto the one engine this build has: the gfx950 HIP kernels on the
    current device, with fp16 weights on MFMA and fp32 accumulation. ``device`` and
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
        self.stats = {"windows": 0, "needs_fallback": 0, "no_speech_skips": 0}

    def transcribe(self, audio, beam_size: int = 1, language: str = "en", **_ignored):
        if beam_size != 1:
            raise NotImplementedError("janus_amd decodes greedily (beam_size=1, transcriber.py:55)")
        if language not in (None, "en"):
            raise NotImplementedError("*.en models transcribe English only (transcriber.py:56)")
        if isinstance(audio, str):
            audio = read_wav_16k(audio)
        audio = np.ascontiguousarray(audio, dtype=np.float32)
        st = generate_segments(self.engine, [audio])[0]
        self._count(st)
        info = TranscriptionInfo("en", 1.0, len(audio) / 16000.0)
        return iter(st.segments), info

    def _count(self, st):
        self.stats["windows"] += st.windows
        self.stats["needs_fallback"] += st.fallbacks
        self.stats["no_speech_skips"] += st.skips


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
        """Batched extension: 48 kHz buffers (any length) -> transcripts, the seek loops
        of all buffers advanced together (one GPU batch per round)."""
        auds = [np.ascontiguousarray(np.asarray(b, dtype=np.float32)[::3]) for b in buffers]
        streams = generate_segments(self.model.engine, auds)
        for st in streams:
            self.model._count(st)
        return [' '.join(s.text.strip() for s in st.segments).strip() for st in streams]


__all__ = ["Transcriber", "WhisperModel", "Segment", "TranscriptionInfo", "read_wav_16k",
           "generate_segments", "split_window", "compression_ratio", "gates", "nat"]
