"""ORACLE — test infrastructure only (see oracle/__init__.py).

Restatements of the reference's host-side decode helpers:
* ``prompt_tag`` — the prosody -> emotion-tag rules of synthesizer.py:149-177, written
  as the reference's if/elif chain (pinned by test_synthesis.py:159-226).
* ``morse`` — synthesizer.py:257-326 (pinned by test_synthesis.py:237-276: "SOS" lasts
  between 2 and 5 s), sample-by-sample with Python math.
* ``ducking`` — engine.py:94-134 gain on int16 PCM.
"""
import math

import numpy as np

MORSE = {'A': '.-', 'B': '-...', 'C': '-.-.', 'D': '-..', 'E': '.', 'F': '..-.', 'G': '--.',
         'H': '....', 'I': '..', 'J': '.---', 'K': '-.-', 'L': '.-..', 'M': '--', 'N': '-.',
         'O': '---', 'P': '.--.', 'Q': '--.-', 'R': '.-.', 'S': '...', 'T': '-', 'U': '..-',
         'V': '...-', 'W': '.--', 'X': '-..-', 'Y': '-.--', 'Z': '--..', '0': '-----',
         '1': '.----', '2': '..---', '3': '...--', '4': '....-', '5': '.....', '6': '-....',
         '7': '--...', '8': '---..', '9': '----.', ' ': ' '}


def prompt_tag(override, prosody):
    if override and override != "Auto":
        return override
    prosody = prosody or {}
    pitch = prosody.get('pitch', 'Normal')
    energy = prosody.get('energy', 'Normal')
    if pitch == 'High' and energy == 'Loud':
        return "excited"
    if pitch == 'High' and energy == 'Normal':
        return "joyful"
    if pitch == 'High' and energy in ('Quiet', 'Low'):
        return "whispering"
    if pitch == 'Low' and energy == 'Loud':
        return "shouting"
    if pitch == 'Low' and energy == 'Low':
        return "sad"
    if pitch == 'Low' and energy == 'Normal':
        return "relaxed"
    if energy == 'Loud':
        return "shouting"
    if energy in ('Quiet', 'Low'):
        return "whispering"
    return "relaxed"


def morse(text, sr=48000, freq=800):
    out = []
    up = text.upper()
    for ch in up:
        if ch not in MORSE:
            continue
        pat = MORSE[ch]
        if pat == ' ':
            out.extend([0] * int(0.7 * sr))
            continue
        for i, sym in enumerate(pat):
            dur = 0.1 if sym == '.' else 0.3
            n = int(dur * sr)
            step = dur / n
            for k in range(n):
                out.append(int(math.sin(2 * math.pi * freq * (k * step)) * 32767 * 0.5))
            if i < len(pat) - 1:
                out.extend([0] * int(0.1 * sr))
        if ch != up[-1]:
            out.extend([0] * int(0.3 * sr))
    return np.array(out, np.int16).tobytes()
