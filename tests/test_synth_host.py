"""Host-side decode helpers (CPU): prompt mapping (backend/tests/test_synthesis.py:159-226),
Morse PCM (test_synthesis.py:237-276) byte-identical to the oracle, WAV framing
(test_e2e_local.py:79-101)."""
import struct

import numpy as np
import pytest

from janus_amd.common.protocol import JanusMode, JanusPacket
from janus_amd.services.synthesizer import Synthesizer, emotion_prompt
from janus_amd.vocoder import emotion_id, wav_bytes
from oracle import synth as osy


def host_synth():
    s = Synthesizer.__new__(Synthesizer)  # no GPU: host-only methods
    s.morse_code_dict = dict(osy.MORSE)
    return s


def test_prompt_override():
    p = JanusPacket("Hello world", JanusMode.SEMANTIC_VOICE, {'energy': 'Normal', 'pitch': 'Normal'},
                    override_emotion="excited")
    prompt, tag = emotion_prompt(p)
    assert prompt.startswith('(excited)') and 'Hello world' in prompt


@pytest.mark.parametrize("pitch", ['High', 'Normal', 'Low', 'Deep', None])
@pytest.mark.parametrize("energy", ['Loud', 'Normal', 'Quiet', 'Low', None])
def test_prompt_mapping_all_pairs(pitch, energy):
    pros = {}
    if energy:
        pros['energy'] = energy
    if pitch:
        pros['pitch'] = pitch
    p = JanusPacket("Test", JanusMode.SEMANTIC_VOICE, pros, override_emotion="Auto")
    prompt, tag = emotion_prompt(p)
    assert tag == osy.prompt_tag("Auto", pros)
    assert prompt == f"({tag}) Test"


def test_prompt_kats():
    for pros, tag in [({'energy': 'Loud', 'pitch': 'High'}, 'excited'),
                      ({'energy': 'Normal', 'pitch': 'High'}, 'joyful'),
                      ({'energy': 'Normal', 'pitch': 'Low'}, 'relaxed')]:
        assert emotion_prompt(JanusPacket("Test", 0, pros, "Auto"))[1] == tag
    # the live engine's override is the str-enum "auto" -> "(auto) text" 
    assert emotion_prompt(JanusPacket("Hi", 0, {}, "auto"))[0] == "(auto) Hi"


@pytest.mark.parametrize("text", ["SOS", "Hello World 42", "", "a a", "ee", "??", "Janus 300bps"])
def test_morse_bytes_match_oracle(text):
    assert host_synth()._generate_morse_audio(text) == osy.morse(text)


def test_morse_sos_duration():
    n = len(host_synth()._generate_morse_audio("SOS")) // 2
    assert 2.0 < n / 48000 < 5.0


def test_wav_layout():
    pcm = (np.arange(100) - 50).astype(np.int16)
    b = wav_bytes(pcm, 44100)
    assert len(b) == 44 + 200
    riff, size, wave_, fmt, sub1, afmt, ch, sr, brate, align, bits, data, dsize = \
        struct.unpack('<4sI4s4sIHHIIHH4sI', b[:44])
    assert (riff, wave_, fmt, data) == (b'RIFF', b'WAVE', b'fmt ', b'data')
    assert (size, sub1, afmt, ch, sr, brate, align, bits, dsize) == (236, 16, 1, 1, 44100, 88200, 2, 16, 200)
    assert np.array_equal(np.frombuffer(b[44:], '<i2'), pcm)


def test_emotion_ids_stable():
    assert emotion_id("relaxed") == 0 and emotion_id("Excited") == 1
    a, b = emotion_id("auto"), emotion_id("panicked")
    assert 6 <= a < 16 and 6 <= b < 16 and emotion_id("auto") == a
