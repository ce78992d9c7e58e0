"""Speech synthesis — drop-in for backend/services/synthesizer.py on MI355X.

Same constructor, routing and private methods as the reference (synthesizer.py:28-326):
``synthesize`` routes MORSE -> ``_generate_morse_audio``, TEXT_ONLY ->
``_generate_fast_tts``, SEMANTIC -> ``_generate_semantic_audio`` with the identical
prosody -> emotion-tag prompt mapping (:149-177) and fallbacks (:205-207, :253-255).

The reference's cloud client is replaced by a module-level ``FishAudio`` with the SDK's
call shape — ``FishAudio(api_key=...)`` (:46) and ``client.tts.convert(text=prompt,
format="wav", latency="balanced", references=[ReferenceAudio(audio=..., text="")] |
reference_id=...)`` (:191-202, :237-251) — backed by the local Firefly-GAN vocoder on the
GPU. It returns WAV bytes (44-byte RIFF header + int16 PCM @ 44.1 kHz, the format the
reference requests). The prompt's leading "(tag)" selects the emotion row, the rest of
the prompt drives the text front end, and the voice follows the SDK arguments: a
``ReferenceAudio`` recording (the hot-reloaded voice-cloning file, :67-104, :183-187) is
embedded on the GPU (janus_vocoder_speaker), a ``reference_id`` selects a stock voice
row, neither means no voice term. Tests patch ``FishAudio`` exactly as the reference
suite does (backend/tests/test_synthesis.py:28-312). Morse generation is host numpy, as
in the reference.
"""
import dataclasses
import hashlib
import logging
import os

import numpy as np

from ..common import wavio
from ..common.protocol import JanusMode, JanusPacket
from ..vocoder import (DEFAULT_REFERENCE_ID, FRAMES_PER_BYTE, VocoderEngine, emotion_id,
                       split_prompt, wav_bytes)

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
        tag = f"{override}"  # f-string, as :152 formats it (a str-enum gives its value)
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


@dataclasses.dataclass
class ReferenceAudio:
    """fishaudio.types.ReferenceAudio's fields as the reference fills them (:184-187)."""
    audio: bytes
    text: str = ""


class _TTS:
    """``client.tts``: ``convert(text=..., format="wav", latency=..., references=...,
    reference_id=...)`` -> WAV bytes rendered by the local GPU vocoder."""

    def __init__(self, engine: VocoderEngine):
        self.engine = engine
        self._ref_key = None     # (len, blake2b) of the last reference recording
        self._ref_voice = None   # its voice vector, or None when it could not be used

    def _recording_voice(self, audio: bytes):
        """Voice vector of a reference recording, computed once per distinct file content
        (the Synthesizer hands the same hot-reloaded bytes with every packet). A recording
        this host cannot decode (MP3 / WebM need FFmpeg) or embed is logged and the packet
        is rendered without the voice term, instead of failing the render: the cloud the
        reference calls accepts those files (synthesizer.py:179-203)."""
        key = (len(audio), hashlib.blake2b(audio, digest_size=16).digest())
        if key != self._ref_key:
            try:
                self._ref_voice = self.engine.speaker_embedding([wavio.read_wav_16k(audio)])[0]
            except Exception as e:
                logger.warning(f"reference audio not usable for voice cloning ({e}); "
                               "rendering without it")
                self._ref_voice = None
            self._ref_key = key
        return self._ref_voice

    def voice(self, references=None, reference_id=None):
        """[latent] f32 voice vector (device) for the SDK's voice arguments, or None."""
        eng = self.engine
        if references:
            ref = references[0]
            audio = ref.audio if isinstance(ref, ReferenceAudio) else ref["audio"]
            return self._recording_voice(bytes(audio))
        if reference_id:
            return eng.voice(reference_id)
        return None

    def convert(self, *, text: str, format: str = "wav", latency: str = "balanced",
                references=None, reference_id=None, **_kw) -> bytes:
        if format != "wav":
            raise ValueError(f"local TTS renders WAV only, not {format!r}")
        tag, _ = split_prompt(text)
        eng = self.engine
        pb = text.encode("utf-8")
        frames = max(1, len(pb)) * FRAMES_PER_BYTE
        v = self.voice(references, reference_id)
        spk = v.reshape(1, -1) if v is not None else None
        lat = eng.frontend([pb], [emotion_id(tag or "relaxed", eng.cfg.n_emotions)], frames, spk)
        _, pcm = eng.forward(lat)
        return wav_bytes(pcm[0].cpu().numpy())


class FishAudio:
    """Module-level stand-in for ``fishaudio.FishAudio`` (synthesizer.py:16, :46): the same
    constructor and ``.tts.convert`` surface over the GPU vocoder. ``api_key`` is kept and
    unused (nothing leaves the machine). Raises if no GPU / HIP library is present."""

    def __init__(self, api_key: str = None, engine: VocoderEngine = None):
        self.api_key = api_key
        self.tts = _TTS(engine if engine is not None else VocoderEngine())


def morse_audio(text: str) -> bytes:
    """Synthesizer._generate_morse_audio without building a Synthesizer (no vocoder)."""
    class _Codes:
        morse_code_dict = MORSE_CODE
    return Synthesizer._generate_morse_audio(_Codes(), text)


class Synthesizer:
    def __init__(self, api_key: str, reference_audio_path: str | None = None):
        self.client = FishAudio(api_key=api_key)
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

    def _generate_semantic_audio(self, packet: JanusPacket) -> bytes:
        """synthesizer.py:133-207."""
        self._check_and_reload_reference_audio()
        prompt, _ = emotion_prompt(packet)
        try:
            references = None
            reference_id = None
            if self.reference_audio_bytes:
                references = [ReferenceAudio(audio=self.reference_audio_bytes, text="")]
            else:
                reference_id = DEFAULT_REFERENCE_ID
            api_params = {"text": prompt, "format": "wav", "latency": "balanced"}
            if references:
                api_params["references"] = references
            else:
                api_params["reference_id"] = reference_id
            return self.client.tts.convert(**api_params)
        except Exception as e:
            logger.error(f"Synthesis error: {e}")
            return self._generate_fast_tts(packet.text, packet.override_emotion)

    def _generate_fast_tts(self, text: str, emotion: str | None = None) -> bytes:
        """synthesizer.py:209-255."""
        self._check_and_reload_reference_audio()
        if emotion and emotion != "Auto":
            prompt = f"({emotion}) {text}"
        else:
            prompt = text
        try:
            api_params = {"text": prompt, "format": "wav", "latency": "balanced"}
            if self.reference_audio_bytes:
                api_params["references"] = [ReferenceAudio(audio=self.reference_audio_bytes, text="")]
            else:
                api_params["references"] = None
            return self.client.tts.convert(**api_params)
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
