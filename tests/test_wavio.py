"""WAV decoding for transcribe_file and the voice-cloning recording: integer
PCM 8/16/24/32-bit, IEEE float 32/64, WAVE_FORMAT_EXTENSIBLE, multi-channel, odd-sized
chunks before the data; compressed files raise ValueError (callers fall back)."""
import struct
import wave

import numpy as np
import pytest

from janus_amd.common.wavio import read_wav_16k, wav_to_f32


def _riff(fmt_tag, ch, sr, bits, payload, extensible=False, extra_chunk=False):
    align = ch * bits // 8
    if extensible:
        fmt = struct.pack("<HHIIHHHHI", 0xFFFE, ch, sr, sr * align, align, bits, 22, bits, 0)
        fmt += struct.pack("<H", fmt_tag) + b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
    else:
        fmt = struct.pack("<HHIIHH", fmt_tag, ch, sr, sr * align, align, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt
    if extra_chunk:
        body += b"LIST" + struct.pack("<I", 3) + b"abc" + b"\x00"   # odd size + pad byte
    body += b"data" + struct.pack("<I", len(payload)) + payload
    return b"RIFF" + struct.pack("<I", len(body)) + body


def test_formats_decode_to_the_same_signal():
    rng = np.random.default_rng(0)
    x = np.clip(rng.standard_normal(1000) * 0.2, -0.99, 0.99)
    i16 = np.round(x * 32767).astype("<i2")
    ref16 = i16.astype(np.float32) / 32768.0
    cases = {
        "pcm16": _riff(1, 1, 16000, 16, i16.tobytes()),
        "pcm16_ext_list": _riff(1, 1, 16000, 16, i16.tobytes(), extensible=True, extra_chunk=True),
        "pcm24": _riff(1, 1, 16000, 24, b"".join((int(v) * 256).to_bytes(3, "little", signed=True)
                                                  for v in i16)),
        "pcm32": _riff(1, 1, 16000, 32, (i16.astype("<i4") << 16).tobytes()),
        "f32": _riff(3, 1, 16000, 32, ref16.astype("<f4").tobytes()),
        "f64_ext": _riff(3, 1, 16000, 64, ref16.astype("<f8").tobytes(), extensible=True),
        "stereo16": _riff(1, 2, 16000, 16, np.repeat(i16, 2).tobytes()),
    }
    for k, data in cases.items():
        y, sr = wav_to_f32(data)
        assert sr == 16000 and y.dtype == np.float32, k
        assert np.array_equal(y, ref16), k
    u8 = _riff(1, 1, 16000, 8, (np.round(x * 127) + 128).astype(np.uint8).tobytes())
    y, _ = wav_to_f32(u8)
    assert np.abs(y - x).max() < 1.0 / 64


def test_matches_wave_module_and_resamples(tmp_path):
    x = (np.sin(np.arange(4800) * 0.01) * 20000).astype("<i2")
    path = tmp_path / "a.wav"
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(48000)
        w.writeframes(x.tobytes())
    y = read_wav_16k(str(path))
    assert np.array_equal(y, (x.astype(np.float32) / 32768.0)[::3])


@pytest.mark.parametrize("data", [b"ID3\x04\x00" + b"\x00" * 64, b"RIFF\x10\x00\x00\x00WAVEjunk",
                                  _riff(2, 1, 16000, 4, b"\x00" * 32)])
def test_unsupported_raise_value_error(data):
    with pytest.raises(ValueError):
        wav_to_f32(data)
