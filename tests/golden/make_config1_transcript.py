"""Generates tests/golden/config1_transcript.json (run from the repo root; ~75 s of CPU).

BASELINE config 1: one 5 s 16 kHz mono utterance through the reference's
``Transcriber('tiny.en').transcribe_file`` (/root/reference/backend/services/
transcriber.py:66-91: faster-whisper ``transcribe(path, beam_size=1, language='en')``
with every other option at its default, so the temperature fallback is on). The expected
transcript is the oracle's restatement of faster-whisper's ``generate_segments`` +
``generate_with_fallback`` (oracle/whisper.py transcribe_segments, pinned to transformers)
on the same seeded synthetic tiny.en weights (seed 0, what ``Transcriber`` loads when no
checkpoint is configured) and the same audio (janus_amd.workload.synth_speech(5, 5.0,
sr=16000), written as 16-bit PCM by the test). Stored: the segments (start, end, text,
tokens), the loop's counters and the joined text transcribe_file returns.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from janus_amd.tokenizer import load_tokenizer  # noqa: E402
from janus_amd.whisper import CONFIGS, mel_filters, synthetic_weights  # noqa: E402
from janus_amd.workload import synth_speech  # noqa: E402
from oracle import whisper as ow  # noqa: E402

OUT = os.path.join(os.path.dirname(__file__), "config1_transcript.json")


def audio():
    """The 16 kHz samples the test's WAV file holds (int16 round trip, as read back)."""
    x = synth_speech(5, 5.0, sr=16000)
    q = (x * 32768).astype("<i2")
    return x, q.astype(np.float32) / 32768.0


def main():
    cfg = CONFIGS["tiny.en"]
    W = synthetic_weights(cfg, 0)
    tk = load_tokenizer()
    _, a = audio()
    segs, cnt = ow.transcribe_segments(a, W, cfg, tk, mel_filters())
    text = " ".join(s[2].strip() for s in segs).strip()
    json.dump({"model": "tiny.en", "weights_seed": 0, "audio": "synth_speech(5, 5.0, sr=16000)",
               "segments": [[float(s[0]), float(s[1]), s[2], [int(t) for t in s[3]]] for s in segs],
               "counters": cnt, "text": text}, open(OUT, "w"), indent=1)
    print(OUT, cnt, repr(text))


if __name__ == "__main__":
    main()
