"""Speech synthesis — drop-in for backend/services/synthesizer.py on MI355X.

Same constructor, routing and private methods as the reference (synthesizer.py:28-326):
``synthesize`` routes MORSE -> ``_generate_morse_audio``, TEXT_ONLY ->
``_generate_fast_tts``, SEMANTIC -> ``_generate_semantic_audio`` with the identical
prosody -> emotion-tag prompt mapping (:149-177) and fallbacks (:205-207, :253-255).
Where the reference calls the Fish Audio cloud (``client.tts.convert``, :202, :251),
this calls the local Firefly-GAN vocoder on the GPU and returns WAV bytes (44-byte
RIFF header + int16 PCM @ 44.1 kHz), the format the reference requests
(``format="wav"``). Voice-cloning reference audio is loaded and hot-reloaded exactly
as in the reference (:67-104) but does not condition the local vocoder.
Morse generation is host numpy, as in the reference.
"""
import logging
import os

import numpy as np

from ..common.protocol import JanusMode, JanusPacket
from ..vocoder import FRAMES_PER_BYTE, VocoderEngine, emotion_id, wav_bytes

logger = logging.getLogger(__name__)

SAMPLE_RATE = 48000  # Hz (synthesizer.py:24; Morse path)
MORSE_FREQUENCY = 800  # Hz


# (pitch, energy) -> tag rules of synthesizer.py:155-175 that look at both tags; every
# other combination falls through to the energy-only rules (:170-175).
_BOTH_TAGS = {
    ('High', 'Loud'): "excited", ('High', 'Normal'): "joyful",
    ('High', 'Quiet'): "whispering", ('High', 'Low'): "whispering",
    ('Low', 'Loud'): "shouting", ('Low', 'Low'): "sad", ('Low', 'Normal'): "relaxed",
}
_ENERGY_ONLY = {'Loud': "shouting", 'Quiet': "whispering", 'Low': "whispering"}


def emotion_prompt(packet: JanusPacket) -> tuple:
    """(prompt, tag) as synthesizer.py:149-177 builds it: a non-"Auto" override wins,
    else the prosody tags pick the emotion. (Prosody emits 'Deep', never 'Low', so deep
    voices reach the energy-only rules, as in the reference.)"""
    override = packet.override_emotion
    if override and override != "Auto":
        tag = str(override)
    else:
        p = packet.prosody or {}
        key = (p.get('pitch', 'Normal'), p.get('energy', 'Normal'))
        tag = _BOTH_TAGS.get(key) or _ENERGY_ONLY.get(key[1], "relaxed")
    return f"({tag}) {packet.text}", tag


MORSE_CODE = {  # synthesizer.py:57-65
    'A': '.-', 'B': '-...', 'C': '-.-.', 'D': '-..', 'E': '.', 'F': '..-.',
    'G': '--.', 'H': '....', 'I': '..', 'J': '.---', 'K': '-.-', 'L': '.-..',
    'M': '--', 'N': '-.', 'O': '---', 'P': '.--.', 'Q': '--.-', 'R': '.-.',
    'S': '...', 'T': '-', 'U': '..-', 'V': '...-', 'W': '.--', 'X': '-..-',
    'Y': '-.--', 'Z': '--..',
    '0': '-----', '1': '.----', '2': '..---', '3': '...--', '4': '....-',
    '5': '.....', '6': '-....', '7': '--...', '8': '---..', '9': '----.',
    ' ': ' ',
}


def morse_audio(text: str) -> bytes:
    """Synthesizer._generate_morse_audio without building a Synthesizer (no vocoder)."""
    class _Codes:
        morse_code_dict = MORSE_CODE
    return Synthesizer._generate_morse_audio(_Codes(), text)


class Synthesizer:
    def __init__(self, api_key: str, reference_audio_path: str | None = None):
        self.api_key = api_key
        self.client = VocoderEngine()
        self.reference_audio_bytes = None
        self._reference_audio_mtime = None
        self._reference_audio_path = reference_audio_path
        if self._reference_audio_path:
            self._load_reference_audio(self._reference_audio_path)
        self.morse_code_dict = dict(MORSE_CODE)

    def _load_reference_audio(self, audio_path: str) -> None:
        try:
            if os.path.exists(audio_path):
                with open(audio_path, 'rb') as f:
                    self.reference_audio_bytes = f.read()
                self._reference_audio_mtime = os.path.getmtime(audio_path)
            else:
                self.reference_audio_bytes = None
                self._reference_audio_mtime = None
        except Exception as e:
            logger.warning(f"Could not load reference audio from {audio_path}: {e}")
            self.reference_audio_bytes = None
            self._reference_audio_mtime = None

    def _check_and_reload_reference_audio(self) -> None:
        if self._reference_audio_path:
            if os.path.exists(self._reference_audio_path):
                current_mtime = os.path.getmtime(self._reference_audio_path)
                if self._reference_audio_mtime is None or self._reference_audio_mtime != current_mtime:
                    self._load_reference_audio(self._reference_audio_path)

    def synthesize(self, packet: JanusPacket) -> bytes:
        if packet.mode == JanusMode.MORSE_CODE:
            return self._generate_morse_audio(packet.text)
        elif packet.mode == JanusMode.TEXT_ONLY:
            return self._generate_fast_tts(packet.text, packet.override_emotion)
        elif packet.mode == JanusMode.SEMANTIC_VOICE:
            return self._generate_semantic_audio(packet)
        else:
            raise ValueError(f"Unknown packet mode: {packet.mode}")

    def _vocode(self, prompt: str, tag: str) -> bytes:
        pb = prompt.encode("utf-8")
        frames = max(1, len(pb)) * FRAMES_PER_BYTE
        lat = self.client.frontend([pb], [emotion_id(tag, self.client.cfg.n_emotions)], frames)
        _, pcm = self.client.forward(lat)
        return wav_bytes(pcm[0].cpu().numpy())

    def _generate_semantic_audio(self, packet: JanusPacket) -> bytes:
        self._check_and_reload_reference_audio()
        prompt, tag = emotion_prompt(packet)
        try:
            return self._vocode(prompt, tag)
        except Exception as e:
            logger.error(f"Synthesis error: {e}")
            return self._generate_fast_tts(packet.text, packet.override_emotion)

    def _generate_fast_tts(self, text: str, emotion: str | None = None) -> bytes:
        self._check_and_reload_reference_audio()
        if emotion and emotion != "Auto":
            prompt, tag = f"({emotion}) {text}", str(emotion)
        else:
            prompt, tag = text, "relaxed"
        try:
            return self._vocode(prompt, tag)
        except Exception as e:
            logger.error(f"Fast TTS error: {e}")
            return b''

    def _generate_morse_audio(self, text: str) -> bytes:
        """synthesizer.py:257-326 at 48 kHz: dot 0.1 s / dash 0.3 s of 800 Hz at half
        scale (truncated to int16), 0.1 s between symbols, 0.7 s for a space, and a 0.3 s
        letter gap that is skipped after ANY character equal to the text's last one
        (the reference compares characters, not positions)."""
        def tone(sec):
            n = int(sec * SAMPLE_RATE)
            ph = 2 * np.pi * MORSE_FREQUENCY * np.linspace(0, sec, n, False)
            return (np.sin(ph) * 32767 * 0.5).astype(np.int16)

        def gap(sec):
            return np.zeros(int(sec * SAMPLE_RATE), dtype=np.int16)

        up = text.upper()
        parts = []
        for ch in up:
            code = self.morse_code_dict.get(ch)
            if code is None:
                continue
            if code == ' ':
                parts.append(gap(0.7))
                continue
            for k, sym in enumerate(code):
                if sym not in '.-':
                    continue
                parts.append(tone(0.1 if sym == '.' else 0.3))
                if k < len(code) - 1:
                    parts.append(gap(0.1))
            if ch != up[-1]:
                parts.append(gap(0.3))
        return (np.concatenate(parts) if parts else np.zeros(0, np.int16)).tobytes()
