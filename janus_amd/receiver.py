"""Receiver decode glue on the GPU.

The reference receiver (backend/services/engine.py:137-312) reads length-prefixed packets
(:201-218), deserializes (:220), synthesizes WAV bytes per packet (:280 ->
Synthesizer.synthesize) and, on playback, ducks the int16 samples while the local user
talks (apply_ducking_if_needed, :94-134). ``ReceiverBatch`` does the same for a batch of
packets drained from any number of connections: one MessagePack decode per packet on the
host, ONE front-end + vocoder pass for all SEMANTIC / TEXT_ONLY packets (JanusPipeline.decode),
the ducking gain in place on the GPU PCM (janus_duck_pcm16) and the 44-byte RIFF framing
(vocoder.wav_bytes, the layout of test_e2e_local.py:79-101). Morse packets stay on the host
(synthesizer.py:257-326), as in the pipeline.
"""
import numpy as np
import torch

from . import _native as nat
from .common.protocol import JanusMode, JanusPacket
from .common.wire import FrameReader
from .services.synthesizer import morse_audio
from .vocoder import wav_bytes


def _duck_level(state):
    """The gain apply_ducking_if_needed would use, or None when it passes audio through."""
    if not getattr(state, "ducking_enabled", True):
        return None
    if not getattr(state, "is_talking", False):
        return None
    level = float(getattr(state, "ducking_level", 0.25))
    if level <= 0.0:
        level = 0.0
    elif level >= 1.0:
        return None
    return level


def duck_pcm16_(pcm: torch.Tensor, level: float) -> torch.Tensor:
    """In place on an int16 GPU tensor: numpy's clip(s.astype(f32) * level).astype(int16)."""
    assert pcm.is_cuda and pcm.dtype == torch.int16 and pcm.is_contiguous()
    nat.call("janus_duck_pcm16", pcm.data_ptr(), pcm.numel(), float(np.float32(level)),
             nat.stream_ptr(pcm.device))
    return pcm


def apply_ducking_if_needed(audio_bytes: bytes, state) -> bytes:
    """Same signature and behaviour as engine.py:94-134 (int16 PCM bytes in and out).
    The reference catches any exception and returns the input unchanged (:132-134)."""
    try:
        level = _duck_level(state)
        if level is None or not audio_bytes:
            return audio_bytes
        samples = np.frombuffer(audio_bytes, dtype=np.int16)
        if samples.size == 0:
            return audio_bytes
        dev = nat.require_gpu()
        t = torch.from_numpy(samples.copy()).to(dev)
        duck_pcm16_(t, level)
        return t.cpu().numpy().tobytes()
    except Exception:
        return audio_bytes


class ReceiverBatch:
    """Batched receiver: feed() raw TCP bytes (any slicing), synthesize() everything that
    completed, returning WAV bytes per packet (b'' for a corrupt packet, engine.py:219-223)."""

    def __init__(self, pipeline, frames: int, state=None):
        self.pipe, self.frames, self.state = pipeline, frames, state
        self.reader = FrameReader()
        self.pending = []

    def feed(self, data: bytes) -> int:
        self.pending.extend(self.reader.feed(data))
        return len(self.pending)

    def synthesize(self):
        raw, self.pending = self.pending, []
        pkts = []
        for b in raw:
            try:
                pkts.append(JanusPacket.deserialize(b))
            except Exception:
                pkts.append(None)
        out = [b""] * len(pkts)
        neural = [i for i, p in enumerate(pkts) if p is not None and p.mode != JanusMode.MORSE_CODE]
        morse = [i for i, p in enumerate(pkts) if p is not None and p.mode == JanusMode.MORSE_CODE]
        level = _duck_level(self.state) if self.state is not None else None
        if neural:
            wav, pcm, _ = self.pipe.decode([raw[i] for i in neural], self.frames)
            if level is not None:
                duck_pcm16_(pcm, level)
            host = pcm.cpu().numpy()
            for k, i in enumerate(neural):
                out[i] = wav_bytes(host[k])
        for i in morse:
            audio = morse_audio(pkts[i].text)
            out[i] = apply_ducking_if_needed(audio, self.state) if self.state is not None else audio
        return out
