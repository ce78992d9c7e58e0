"""Phrase segmentation (engine.py:438-506) against the oracle restatement, host only."""
import numpy as np
import pytest

from janus_amd.streaming import CHUNK, PhraseSegmenter
from oracle.segmenter import segment


def run_product(chunks, speech, recording, streaming, non_vad):
    seg = PhraseSegmenter()
    out = []
    for i, c in enumerate(chunks):
        p = seg.push(c, speech[i], streaming=streaming[i], recording=recording[i], non_vad_mode=non_vad[i])
        if p is not None:
            out.append((i, p))
    return out


@pytest.mark.parametrize("seed", range(12))
def test_segmenter_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    n = 600
    chunks = [rng.standard_normal(CHUNK).astype(np.float32) * 0.01 + i for i in range(n)]
    # bursts of speech / silence of random lengths (incl. runs of exactly 15/16 silent chunks)
    speech, cur = [], bool(rng.integers(2))
    while len(speech) < n:
        run = int(rng.choice([1, 2, 5, 15, 16, 17, 30, 80]))
        speech += [cur] * run
        cur = not cur
    speech = speech[:n]
    recording = [False] * n
    streaming = [True] * n
    non_vad = [False] * n
    if seed % 3 == 1:   # push-to-talk holds
        for a in rng.integers(0, n - 40, 4):
            for k in range(int(a), int(a) + int(rng.integers(1, 30))):
                recording[k] = True
    if seed % 3 == 2:   # streaming toggled off, non-VAD (Morse/Text) mode stretches
        for a in rng.integers(0, n - 40, 3):
            for k in range(int(a), int(a) + 20):
                streaming[k] = False
        for a in rng.integers(0, n - 40, 3):
            for k in range(int(a), int(a) + 10):
                non_vad[k] = True
    got = run_product(chunks, speech, recording, streaming, non_vad)
    ref = segment(chunks, speech, recording, streaming, non_vad)
    assert [i for i, _ in got] == [i for i, _ in ref]
    for (_, a), (_, b) in zip(got, ref):
        assert np.array_equal(a, b)


def test_short_phrase_dropped_and_preroll_kept():
    seg = PhraseSegmenter()
    z = np.zeros(CHUNK, np.float32)
    # 3 silent chunks (pre-roll), 1 speech chunk, 16 silent -> 20 chunks >= 9216: emitted
    for _ in range(3):
        assert seg.push(z, False) is None
    assert seg.push(z + 1, True) is None
    outs = [seg.push(z, False) for _ in range(16)]
    assert outs[-1] is not None and len(outs[-1]) == (3 + 1 + 16) * CHUNK
    # the deque is not cleared by a phrase (engine.py:481): its 3 old chunks + new ones
    seg2 = PhraseSegmenter()
    for _ in range(16):
        seg2.push(z, False)          # fills pre-roll (last 10 kept), counter 16 > 15
    p = seg2.push(z + 1, True)
    assert p is None and len(seg2.audio_buffer) == 11


def test_split_window_faster_whisper_rules():
    """generate_segments' slicing (CPU): consecutive timestamp pairs close segments, a
    single trailing timestamp moves the seek to the window end, otherwise the seek goes to
    the last pair; no timestamps -> one segment of the window (or the last stamp)."""
    from janus_amd.services.transcriber import split_window
    from janus_amd.tokenizer import WhisperTokenizer
    tk = WhisperTokenizer()
    tb = tk.timestamp_begin
    a, b = 400, 500
    # <|0.00|> a <|1.00|><|1.00|> b <|2.00|>  (single ending)
    segs, nseek = split_window(tk, [tb, a, tb + 50, tb + 50, b, tb + 100], 1000, 3000)
    assert [s[2] for s in segs] == [[tb, a, tb + 50], [tb + 50, b, tb + 100]]
    assert segs[0][:2] == (10.0, 11.0) and nseek == 4000
    # trailing partial after the last pair: seek to that pair (1.00 s = 100 frames)
    segs, nseek = split_window(tk, [tb, a, tb + 50, tb + 50, b], 0, 3000)
    assert len(segs) == 1 and nseek == 100
    # no pair: one segment to the last timestamp
    segs, nseek = split_window(tk, [tb + 5, a, b, tb + 75], 0, 2500)
    assert segs == [(0.0, 1.5, [tb + 5, a, b, tb + 75])] and nseek == 2500
    # no timestamps at all: the whole window
    segs, nseek = split_window(tk, [a, b], 300, 1200)
    assert segs == [(3.0, 15.0, [a, b])] and nseek == 1500
    # <|0.00|><|0.00|> would not advance: move on by the window
    segs, nseek = split_window(tk, [tb, tb, a], 0, 3000)
    assert nseek == 3000


def test_gates():
    from janus_amd.services.transcriber import compression_ratio, gates
    assert compression_ratio("ab" * 200) > 2.4
    assert gates("hello there", -0.3, 0.01) == (False, False)
    assert gates("hello there", -2.0, 0.01) == (True, False)        # low log-prob: fallback
    assert gates("ab" * 200, -0.3, 0.01) == (True, False)            # repetitive: fallback
    assert gates("hello there", -2.0, 0.9) == (False, True)         # silence: skip, no fallback
    assert gates("hello there", -0.5, 0.9) == (False, False)        # confident text: keep


def test_silero_oracle_basis_and_state():
    """The silero STFT basis is the Hann-windowed DFT (a 1 kHz tone peaks in bin 16 of
    256 at 16 kHz); the oracle model is deterministic and stateful across calls."""
    import torch.nn.functional as F
    import torch
    from janus_amd.services.vad import stft_basis, synthetic_weights
    from oracle.vad import OracleSilero
    b = stft_basis()
    t = np.sin(2 * np.pi * 1000 * np.arange(256) / 16000).astype(np.float32)
    mag = np.hypot(b[:129] @ t, b[129:] @ t)
    assert int(np.argmax(mag)) == 16
    W = synthetic_weights(seed=1)
    a, c = OracleSilero(W), OracleSilero(W)
    chunk = np.random.default_rng(0).standard_normal(512).astype(np.float32) * 0.1
    p1, p2 = a(chunk), a(chunk)
    assert 0.0 < p1 < 1.0 and p1 != p2          # state carried
    assert c(chunk) == p1                        # deterministic from a fresh state
