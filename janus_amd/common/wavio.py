"""WAV decoding shared by the STT file path (transcriber.py:66-91) and the voice-cloning
reference recording (synthesizer.py:67-88 keeps it as raw file bytes and the cloud decodes
it). A small RIFF reader instead of the `wave` module, which on Python 3.10 rejects float
and WAVE_FORMAT_EXTENSIBLE files: integer PCM of 8 (unsigned), 16, 24 or 32 bits and IEEE
float of 32 or 64 bits, plain or extensible, any channel count (averaged to mono).
Compressed formats (MP3, WebM, ...) need FFmpeg, which this image lacks: they raise
ValueError and the callers decide the fallback."""
import io
import struct

import numpy as np

_PCM, _FLOAT, _EXTENSIBLE = 1, 3, 0xFFFE


def _riff_chunks(data: bytes):
    if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError("not a RIFF/WAVE file")
    pos = 12
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        yield cid, body
        pos += 8 + size + (size & 1)   # chunks are word aligned


def wav_to_f32(src) -> tuple:
    """A path, file object or WAV bytes -> (mono float32 samples, sample rate). Integer
    PCM is scaled by 2^(bits-1) (16-bit: /32768, audio_io.py:125-126), float is taken as
    is."""
    if isinstance(src, (bytes, bytearray, memoryview)):
        data = bytes(src)
    elif isinstance(src, io.IOBase) or hasattr(src, "read"):
        data = src.read()
    else:
        with open(src, "rb") as f:
            data = f.read()
    fmt = raw = None
    for cid, body in _riff_chunks(data):
        if cid == b"fmt ":
            fmt = body
        elif cid == b"data" and raw is None:
            raw = body
    if fmt is None or raw is None or len(fmt) < 16:
        raise ValueError("WAV file without fmt/data chunks")
    tag, ch, sr, _, align, bits = struct.unpack("<HHIIHH", fmt[:16])
    if tag == _EXTENSIBLE:
        if len(fmt) < 26:
            raise ValueError("truncated WAVE_FORMAT_EXTENSIBLE header")
        tag = struct.unpack("<H", fmt[24:26])[0]   # first two bytes of the subformat GUID
    if ch < 1 or align < ch:
        raise ValueError("bad WAV channel layout")
    width = align // ch
    n = len(raw) // align
    raw = raw[:n * align]
    if tag == _PCM and width == 1:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif tag == _PCM and width == 2:
        x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    elif tag == _PCM and width == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / float(1 << 23)
    elif tag == _PCM and width == 4:
        x = (np.frombuffer(raw, "<i4").astype(np.float64) / float(1 << 31)).astype(np.float32)
    elif tag == _FLOAT and width == 4:
        x = np.frombuffer(raw, "<f4").astype(np.float32)
    elif tag == _FLOAT and width == 8:
        x = np.frombuffer(raw, "<f8").astype(np.float32)
    else:
        raise ValueError(f"unsupported WAV encoding (format {tag}, {8 * width} bits)")
    if ch > 1:
        x = x.reshape(-1, ch).mean(axis=1)
    return np.ascontiguousarray(x, np.float32), sr


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
