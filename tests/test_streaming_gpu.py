"""Streaming encode (config 5) and receiver glue on the GPU."""
import math

import numpy as np
import pytest
import torch

from janus_amd.common.wire import frame_batch
from janus_amd.receiver import ReceiverBatch, apply_ducking_if_needed, duck_pcm16_
from janus_amd.streaming import CHUNK, VAD_CENTER_DB, VAD_WIDTH_DB, StreamingEncoder, VoiceActivityDetector
from janus_amd.whisper import CONFIGS, WhisperEngine
from janus_amd.workload import synth_speech
from oracle import packet as opk
from oracle.prosody import OracleProsody
from oracle.segmenter import duck, segment

pytestmark = pytest.mark.gpu


class _State:
    def __init__(self, **kw):
        self.__dict__.update(kw)


@pytest.mark.parametrize("level", [0.0, 0.25, 0.5, 0.999])
def test_duck_bit_exact(gpu, level):
    rng = np.random.default_rng(int(level * 1000))
    s = rng.integers(-32768, 32768, 100003, dtype=np.int64).astype(np.int16)
    s[:4] = [-32768, 32767, -1, 1]
    ref = np.frombuffer(duck(s.tobytes(), True, True, level), np.int16)
    t = torch.from_numpy(s.copy()).to(gpu)
    duck_pcm16_(t, level)
    assert np.array_equal(t.cpu().numpy(), ref)
    st = _State(ducking_enabled=True, is_talking=True, ducking_level=level)
    assert apply_ducking_if_needed(s.tobytes(), st) == ref.tobytes()


def test_duck_pass_through(gpu):
    b = np.arange(-50, 50, dtype=np.int16).tobytes()
    assert apply_ducking_if_needed(b, _State(ducking_enabled=False, is_talking=True)) == b
    assert apply_ducking_if_needed(b, _State(ducking_enabled=True, is_talking=False)) == b
    assert apply_ducking_if_needed(b, _State(ducking_enabled=True, is_talking=True, ducking_level=1.5)) == b
    assert apply_ducking_if_needed(b"", _State(ducking_enabled=True, is_talking=True)) == b""


def test_vad_energy(gpu):
    rng = np.random.default_rng(3)
    amp = np.array([0.0, 1e-4, 1e-3, 5e-3, 0.01, 0.1, 0.5], np.float32)
    x = (rng.standard_normal((len(amp), CHUNK)).astype(np.float32) * amp[:, None]).astype(np.float32)
    vad = VoiceActivityDetector()
    prob = vad.probabilities(torch.from_numpy(x).to(gpu)).cpu().numpy()
    ms = (x[:, ::3].astype(np.float64) ** 2).mean(1)
    db = 10 * np.log10(ms + 1e-12)
    ref = 1 / (1 + np.exp(-(db - VAD_CENTER_DB) / VAD_WIDTH_DB))
    assert np.allclose(prob, ref, atol=1e-4)
    assert vad.is_speech(x[-1]) and not vad.is_speech(x[0])


@pytest.fixture(scope="module")
def tiny(gpu):
    return WhisperEngine(CONFIGS["tiny.en"], seed=0)


def _streaming_case(gpu, w, S, ticks, per_tick, mode=None, gap_s=1.0, seed0=300, min_phrases=1,
                    max_length=8, temperatures=None, refs=None):
    from janus_amd.common.protocol import JanusMode
    from janus_amd.services.transcriber import TEMPERATURES
    mode = JanusMode.SEMANTIC_VOICE if mode is None else mode
    enc = StreamingEncoder(S, w, max_length=max_length, mode=mode,
                           temperatures=TEMPERATURES if temperatures is None else temperatures)
    total = ticks * per_tick * CHUNK
    audio = np.zeros((S, total), np.float32)
    for s in range(S):  # speech / silence / speech so phrases complete mid-run
        a = synth_speech(seed0 + s, 2.0)
        b = synth_speech(seed0 + 100 + s, 1.2)
        g = int(gap_s * 48000)
        audio[s, 5000:5000 + len(a)] = a
        audio[s, 5000 + len(a) + g:5000 + len(a) + g + len(b)] = b
    vad = VoiceActivityDetector()
    dec = vad.is_speech_batch(torch.from_numpy(audio.reshape(-1, CHUNK)).to(gpu)).reshape(S, -1)
    non_vad = mode in (JanusMode.TEXT_ONLY, JanusMode.MORSE_CODE)
    got = []
    for t in range(ticks):
        blk = audio[:, t * per_tick * CHUNK:(t + 1) * per_tick * CHUNK]
        got += [(t, r) for r in enc.push(blk, timestamp=1700000000.25)]
    n_ph = 0
    for s in range(S):
        chunks = [audio[s, i * CHUNK:(i + 1) * CHUNK] for i in range(ticks * per_tick)]
        ref = segment(chunks, list(dec[s]), non_vad=[non_vad] * len(chunks))
        mine = [r for _, r in got if r["stream"] == s]
        assert len(mine) == len(ref), (s, len(mine), len(ref))
        if refs is not None:
            refs[s] = [ph for _, ph in ref]
        n_ph += len(ref)
        op = OracleProsody(48000)  # one stateful detector per channel
        for r, (_, ph) in zip(mine, ref):
            tags = op.analyze_buffer(ph)[0]
            assert r["tags"] == tags
            if r["text"].strip():
                assert r["packet"] == opk.serialize(r["text"], int(mode), tags, "auto", 1700000000.25)
            else:
                assert r["packet"] is None
    assert n_ph >= min_phrases
    assert enc.p50_ms() > 0
    return got


def test_streaming_encoder_matches_oracle(gpu, tiny):
    # 320 ms blocks (10 x 1536 @ 48 kHz), 2 channels
    _streaming_case(gpu, tiny, S=2, ticks=14, per_tick=10, min_phrases=2)


def test_streaming_encoder_16_channels(gpu, tiny):
    """Config 5's per-GPU share: 16 channels of 320 ms blocks."""
    _streaming_case(gpu, tiny, S=16, ticks=14, per_tick=10, seed0=700, min_phrases=16)


def test_streaming_16_channels_base_448(gpu):
    """Config 5's per-GPU share at its real decode setting: base.en, max_length 448 (the
    reference's default), 16 channels, T = 0. For channels 0 and 9: every phrase's text
    equals the seek loop (generate_segments) on the oracle segmenter's phrase audio, and
    the first window of every phrase decodes to the oracle's tokens (KV-cached fp32
    decoder on the same encoder output) or diverges first at an oracle near-tie."""
    from janus_amd.services.transcriber import generate_segments
    from janus_amd.whisper import synthetic_weights
    from oracle import whisper as ow
    cfg = CONFIGS["base.en"]
    w = WhisperEngine(cfg, seed=0)
    refs = {}
    # 20 ticks of 320 ms: both phrases of every channel complete (the second needs 15 silent
    # chunks after it)
    got = _streaming_case(gpu, w, S=16, ticks=20, per_tick=10, seed0=900, min_phrases=32,
                          max_length=448, temperatures=(0.0,), refs=refs)
    W = synthetic_weights(cfg, 0)
    tk = w.tokenizer
    plen = len(tk.sot_sequence)
    checked = 0
    for s in (0, 9):
        mine = [r for _, r in got if r["stream"] == s]
        phrases = refs[s]
        auds = [np.ascontiguousarray(ph[::3]) for ph in phrases]
        sts = generate_segments(w, auds, max_length=448, temperatures=(0.0,))
        for r, st in zip(mine, sts):
            assert r["text"] == " ".join(sg.text.strip() for sg in st.segments).strip()
        # first windows: the GPU decoder vs the oracle decoder on the GPU encoder output
        pcm = torch.from_numpy(np.concatenate(phrases + [np.zeros(1, np.float32)])).to(gpu)
        offs = torch.tensor(np.concatenate([[0], np.cumsum([len(p) for p in phrases])]),
                            dtype=torch.int64, device=gpu)
        enc = w.encode(w.logmel(pcm, offs, len(phrases), 3))
        dec = w.decode_ex(enc, max_length=448)
        toks, nt = dec.tokens.cpu().numpy(), dec.n_tokens.cpu().numpy()
        ref = ow.greedy_cached(enc.float().cpu(), W, cfg, tk, 448, no_speech=50361)
        for b, rr in enumerate(ref):
            g = [int(t) for t in toks[b][plen:plen + int(nt[b])]]
            if g != rr["tokens"]:
                first = next((i for i in range(min(len(g), len(rr["tokens"])))
                              if g[i] != rr["tokens"][i]), min(len(g), len(rr["tokens"])))
                margin = rr["margins"][first] if first < len(rr["margins"]) else 0.0
                assert margin < 2e-3, (s, b, first, margin)
            checked += 1
    assert checked >= 4


def test_streaming_two_phrases_one_push(gpu, tiny):
    """One long block completes two phrases on the same channel: the second phrase's YIN
    must continue from the first one's detector state (duplicate channel)."""
    got = _streaming_case(gpu, tiny, S=2, ticks=1, per_tick=160, gap_s=0.8, seed0=500, min_phrases=2)
    per = {}
    for _, r in got:
        per[r["stream"]] = per.get(r["stream"], 0) + 1
    assert max(per.values()) >= 2


def test_streaming_long_phrase_full_seek_loop(gpu, tiny):
    """a phrase longer than one 30 s window (continuous speech, no 0.5 s pause)
    is transcribed by the whole seek loop, as transcribe_buffer does for the engine
    (engine.py:514), not truncated to its first window."""
    from janus_amd.services.transcriber import generate_segments
    enc = StreamingEncoder(1, tiny, max_length=8)
    x = synth_speech(880, 33.0)
    total = (len(x) + 5000 + 48000 + 10 * CHUNK - 1) // (10 * CHUNK) * (10 * CHUNK)
    audio = np.zeros((1, total), np.float32)
    audio[0, 5000:5000 + len(x)] = x
    vad = VoiceActivityDetector()
    dec = vad.is_speech_batch(torch.from_numpy(audio.reshape(-1, CHUNK)).to(gpu)).reshape(1, -1)
    got = []
    for t in range(total // (10 * CHUNK)):
        got += enc.push(audio[:, t * 10 * CHUNK:(t + 1) * 10 * CHUNK])
    chunks = [audio[0, i * CHUNK:(i + 1) * CHUNK] for i in range(total // CHUNK)]
    ref = segment(chunks, list(dec[0]), non_vad=[False] * len(chunks))
    long_refs = [ph for _, ph in ref if (len(ph) + 2) // 3 > 480000]
    assert len(long_refs) == 1 and enc.long_phrases == 1
    st = generate_segments(tiny, [np.ascontiguousarray(long_refs[0][::3])], max_length=8,
                           temperatures=enc.temperatures)[0]
    assert st.windows >= 2
    want = ' '.join(sg.text.strip() for sg in st.segments).strip()
    mine = [r for r in got if r["text"] == want]
    assert len(mine) == 1


def test_streaming_text_only_bypasses_gate(gpu, tiny):
    """TEXT_ONLY / MORSE skip the speech gate (engine.py:473-474): every chunk counts as
    speech, so the whole run is one phrase that never closes on silence."""
    from janus_amd.common.protocol import JanusMode
    enc = StreamingEncoder(1, tiny, max_length=8, mode=JanusMode.TEXT_ONLY)
    blk = np.zeros((1, 40 * CHUNK), np.float32)  # 1.3 s of digital silence
    assert enc.push(blk) == []
    assert len(enc.segmenters[0].audio_buffer) == 40


def test_receiver_batch(gpu):
    from janus_amd.pipeline import JanusPipeline
    from janus_amd.common.protocol import JanusMode, JanusPacket
    pipe = JanusPipeline("tiny.en", max_length=8)
    pk = [JanusPacket("hello there", JanusMode.SEMANTIC_VOICE, {"energy": "Loud", "pitch": "High"}, "Auto", 1.0),
          JanusPacket("sos", JanusMode.MORSE_CODE, {}, "Auto", 2.0),
          JanusPacket("fast one", JanusMode.TEXT_ONLY, {}, "happy", 3.0)]
    raw = [p.serialize() for p in pk]
    stream = frame_batch(raw[:2]) + frame_batch([b"\x93garbage"]) + frame_batch(raw[2:])
    st = _State(ducking_enabled=True, is_talking=True, ducking_level=0.25)
    rb = ReceiverBatch(pipe, 12, st)
    for i in range(0, len(stream), 7):
        rb.feed(stream[i:i + 7])
    out = rb.synthesize()
    assert len(out) == 4 and out[2] == b""
    plain = ReceiverBatch(pipe, 12, None)
    plain.feed(stream)
    ref = plain.synthesize()
    for k in (0, 3):
        assert out[k][:44] == ref[k][:44] and len(out[k]) == 44 + 12 * 512 * 2
        assert out[k][44:] == duck(ref[k][44:], True, True, 0.25)
    assert out[1] == duck(ref[1], True, True, 0.25)


def test_streaming_async_matches_sync(gpu, tiny):
    """Asynchronous ingest (encode on a worker stream) returns the same phrases, tags and
    packets per channel, in order, as the blocking push; the duplex receiver leg renders
    exactly what JanusPipeline.decode renders for those packets."""
    from janus_amd.pipeline import JanusPipeline
    S, ticks, per_tick = 3, 14, 10
    audio = np.zeros((S, ticks * per_tick * CHUNK), np.float32)
    for s in range(S):
        a = synth_speech(800 + s, 2.0)
        b = synth_speech(900 + s, 1.2)
        audio[s, 3000:3000 + len(a)] = a
        audio[s, 3000 + len(a) + 40000:3000 + len(a) + 40000 + len(b)] = b
    rx = JanusPipeline("tiny.en", max_length=8)
    res = {}
    for asyn in (False, True):
        enc = StreamingEncoder(S, tiny, max_length=8, asynchronous=asyn, receiver=rx)
        got = []
        for t in range(ticks):
            got += enc.push(audio[:, t * per_tick * CHUNK:(t + 1) * per_tick * CHUNK], timestamp=7.0)
        got += enc.flush()
        enc.close()
        res[asyn] = got
        assert all(r["latency_s"] > 0 for r in got) and enc.max_queue >= (1 if asyn else 0)
    key = lambda r: (r["stream"], r["text"], tuple(r["tags"].items()), r["packet"])
    a_s, a_a = sorted(map(key, res[False])), sorted(map(key, res[True]))
    assert a_s == a_a and len(a_s) >= 2
    for s in range(S):  # per-channel order preserved
        assert [r["packet"] for r in res[False] if r["stream"] == s] == \
            [r["packet"] for r in res[True] if r["stream"] == s]
    for rs in res.values():
        for r in rs:
            if r["packet"] is not None:
                assert "pcm16" in r and r["pcm16"].dtype == torch.int16


def test_silero_gate_matches_oracle(gpu):
    """The neural gate (csrc/vad.hip, silero-vad v5 graph, seeded weights of the published
    shapes) vs the oracle restatement, 3 channels x 24 capture chunks with per-channel
    state carried across two calls; decisions identical away from the threshold."""
    from janus_amd.services.vad import MultiStreamGate, VoiceActivityDetector, synthetic_weights
    from oracle.vad import OracleSilero
    W = synthetic_weights(seed=4)
    rng = np.random.default_rng(9)
    S, n = 3, 24
    x = np.zeros((S, n, CHUNK), np.float32)
    x[0] = (rng.standard_normal((n, CHUNK)) * 0.1).astype(np.float32)
    x[1] = synth_speech(31, n * CHUNK / 48000.0)[:n * CHUNK].reshape(n, CHUNK)
    x[2, 8:] = (0.3 * np.sin(2 * np.pi * 300 * np.arange(16 * CHUNK) / 48000)).reshape(16, CHUNK)
    gate = MultiStreamGate(S, weights=W)
    assert gate.neural
    d = torch.from_numpy(x).to(gpu)
    p = torch.cat([gate.probabilities(d[:, :10].contiguous()), gate.probabilities(d[:, 10:].contiguous())], 1)
    p = p.cpu().numpy()
    for s in range(S):
        o = OracleSilero(W)
        ref = np.array([o(x[s, j, ::3]) for j in range(n)])
        assert np.abs(p[s] - ref).max() < 1e-5, (s, np.abs(p[s] - ref).max())
        far = np.abs(ref - 0.5) > 1e-4
        assert np.array_equal((p[s] > 0.5)[far], (ref > 0.5)[far])
    # the drop-in single-stream detector: the same state machine, one chunk per call
    det = VoiceActivityDetector(weights=W)
    o = OracleSilero(W)
    for j in range(n):
        pr = o(x[1, j, ::3])
        got = det.is_speech(x[1, j])
        if abs(pr - 0.5) > 1e-4:
            assert got == (pr > 0.5)
