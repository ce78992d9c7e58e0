"""16-bit PCM WAV decoding shared by the STT file path (transcriber.py:66-91) and the
voice-cloning reference recording (synthesizer.py:67-88 keeps it as raw file bytes)."""
import io
import wave

import numpy as np


def wav_to_f32(src) -> tuple:
    """A path or WAV bytes -> (mono float32 samples in [-1, 1), sample rate)."""
    fh = io.BytesIO(src) if isinstance(src, (bytes, bytearray, memoryview)) else src
    with wave.open(fh, "rb") as w:
        sr, ch, sw, n = w.getframerate(), w.getnchannels(), w.getsampwidth(), w.getnframes()
        raw = w.readframes(n)
    if sw != 2:
        raise ValueError("only 16-bit PCM WAV is supported")
    x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0   # audio_io.py:125-126
    if ch > 1:
        x = x.reshape(-1, ch).mean(axis=1)
    return x.astype(np.float32), sr


def to_16k(x: np.ndarray, sr: int) -> np.ndarray:
    """48 kHz by [::3] (transcriber.py:51), 16 kHz as is, other rates by linear
    interpolation."""
    if sr == 16000:
        return np.ascontiguousarray(x, np.float32)
    if sr == 48000:
        return np.ascontiguousarray(x[::3])
    t = np.arange(int(round(len(x) * 16000 / sr))) * (sr / 16000.0)
    return np.interp(t, np.arange(len(x)), x).astype(np.float32)


def read_wav_16k(src) -> np.ndarray:
    x, sr = wav_to_f32(src)
    return to_16k(x, sr)
