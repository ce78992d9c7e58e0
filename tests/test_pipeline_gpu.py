"""End-to-end batched encode/decode on the GPU (engine.py:510-552 -> receiver):
packet bytes bit-identical to the oracle packer given the GPU's text and the oracle's
prosody tags; drop-in Transcriber on a 16 kHz WAV (BASELINE config 1)."""
import wave

import numpy as np
import pytest
import torch

from janus_amd.pipeline import JanusPipeline, ServingTuning
from janus_amd.workload import synth_speech
from oracle import packet as opk
from oracle.prosody import OracleProsody

pytestmark = pytest.mark.gpu


def test_pipeline_small(gpu):
    pipe = JanusPipeline("tiny.en", max_length=12)
    utts = [synth_speech(77 + k, 2.0 + k) for k in range(3)]
    lengths = [len(u) for u in utts]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=gpu)
    pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(gpu)
    res = pipe.encode(pcm, offs, lengths, timestamp=1700000000.5)
    for b, u in enumerate(utts):
        tags = OracleProsody(48000).analyze_buffer(u)[0]
        assert res.tags[b] == tags
        if res.texts[b].strip():
            assert res.packets[b] == opk.serialize(res.texts[b], 0, tags, "auto", 1700000000.5)
        else:
            assert res.packets[b] is None
    wav, pcm16, prompts = pipe.decode(res.packets, 20)
    assert wav.shape[1] == 20 * 512 and len(prompts) == sum(p is not None for p in res.packets)
    assert torch.isfinite(wav).all()


def test_transcriber_wav(gpu, tmp_path):
    from janus_amd.services.transcriber import Transcriber
    x = synth_speech(5, 5.0, sr=16000)
    path = tmp_path / "a.wav"
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes((x * 32768).astype("<i2").tobytes())
    tr = Transcriber("tiny.en")
    t1 = tr.transcribe_file(str(path))
    t2 = tr.transcribe_buffer(np.repeat(x, 3))  # 48 kHz buffer whose [::3] is x
    assert isinstance(t1, str) and t1 == t2
    # BASELINE config 1 against the oracle: faster-whisper's seek loop with its default
    # temperature fallback, restated (oracle/whisper.py transcribe_segments) on the same
    # seeded tiny.en weights and the same int16 samples (tests/golden/
    # make_config1_transcript.py wrote the fixture)
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                       "config1_transcript.json")))
    assert t1 == gold["text"], (t1, gold["text"])
    before = dict(tr.model.stats)
    segs, _ = tr.model.transcribe(str(path), beam_size=1, language="en")
    got = [[s.start, s.end, s.text, list(s.tokens)] for s in segs]
    assert [g[2:] for g in got] == [g[2:] for g in gold["segments"]]
    assert np.allclose([g[:2] for g in got], [g[:2] for g in gold["segments"]])
    for k, ko in (("windows", "windows"), ("needs_fallback", "needs_fallback"),
                  ("no_speech_skips", "skips"), ("fallback_decodes", "fallback_decodes")):
        assert tr.model.stats[k] - before[k] == gold["counters"][ko], k


@pytest.mark.parametrize("yin_dec", [0, 1])
def test_overlapped_step_matches_sequential(gpu, yin_dec):
    """The serving pipeline (encode batch i on the whole GPU, then the greedy decoder of
    batch i and the vocoder of batch i-1 + YIN on disjoint CU-masked streams) produces the
    same packets and the same waveforms as the back-to-back step — with all of YIN on the
    vocoder side (the default) and with the first utterance's YIN on the decoder side
    (yin_dec_utts=1: the prosody result comes back in two parts)."""
    pipe = JanusPipeline("tiny.en", max_length=12, tuning=ServingTuning(yin_dec_utts=yin_dec))
    batches = []
    for i in range(2):
        utts = [synth_speech(300 + 10 * i + k, 1.5 + 0.5 * k) for k in range(3)]
        lengths = [len(u) for u in utts]
        offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=gpu)
        pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(gpu)
        batches.append((pcm, offs, lengths))
    frames = 16
    seq = []
    for pcm, offs, lengths in batches:
        enc = pipe.encode(pcm, offs, lengths, timestamp=5.0)
        wav, pcm16, _ = pipe.decode(enc.packets, frames)
        seq.append((enc.packets, wav, pcm16))
    outs = [pipe.step_overlapped(pcm, offs, lengths, frames, 16, timestamp=5.0)
            for pcm, offs, lengths in batches]
    outs.append(pipe.flush(frames))
    assert outs[0] == (None, None, None)  # nothing pending before the first step
    for i in range(2):
        res, wav, pcm16 = outs[i + 1]  # batch i finishes one step later
        assert res.packets == seq[i][0]
        if seq[i][1] is None:
            assert wav is None
            continue
        torch.testing.assert_close(wav, seq[i][1], rtol=0, atol=0)
        assert torch.equal(pcm16, seq[i][2])


def _batch(gpu, seeds_secs):
    utts = [synth_speech(sd, sec) for sd, sec in seeds_secs]
    lengths = [len(u) for u in utts]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(lengths)]), dtype=torch.int64, device=gpu)
    pcm = torch.from_numpy(np.concatenate(utts + [np.zeros(1, np.float32)])).to(gpu)
    return utts, pcm, offs, lengths


def _same_streams(a, b):
    """Two seek-loop states equal: windows, counters, every window's settled tokens and
    every segment (times, text, tokens)."""
    assert a.windows == b.windows and a.seek == b.seek
    assert (a.fallbacks, a.skips, a.fallback_decodes) == (b.fallbacks, b.skips, b.fallback_decodes)
    assert a.window_tokens == b.window_tokens
    assert [(g.seek, g.start, g.end, g.text, g.tokens) for g in a.segments] == \
        [(g.seek, g.start, g.end, g.text, g.tokens) for g in b.segments]


@pytest.mark.parametrize("sets,voc_dec", [(2, 0), (3, 0), (4, 0), (2, 1), (2, 3)])
def test_staggered_step_matches_sequential(gpu, sets, voc_dec):
    """The continuous-batching serving step (step_staggered: windows enter N slot sets of B
    rows as fresh rows — each batch's first windows, then its clips' continuation windows from
    the seek the previous window ended at — and every decoder call advances all sets;
    N = tuning.stagger_sets) produces, per batch and in order, the same seek loops (windows,
    tokens, segments), packets and waveforms as the back-to-back step of that batch alone;
    flush_staggered drains. With tuning.voc_dec_utts = k the batch's last k packets render on
    the decoder's CUs through a second vocoder context: the waveforms are still
    bit-identical, in packet order."""
    pipe = JanusPipeline("tiny.en", max_length=24, temperatures=(0.0,),
                         tuning=ServingTuning(stagger_sets=sets, voc_dec_utts=voc_dec))
    batches = [_batch(gpu, [(700 + 10 * i + k, 1.5 + 0.5 * k) for k in range(3)])[1:] for i in range(3)]
    frames = 16
    seq = []
    for pcm, offs, lengths in batches:
        enc = pipe.encode(pcm, offs, lengths, timestamp=5.0)
        wav, pcm16, _ = pipe.decode(enc.packets, frames)
        seq.append((enc, wav, pcm16))
    outs = [pipe.step_staggered(pcm, offs, lengths, frames, 16, timestamp=5.0)
            for pcm, offs, lengths in batches]
    assert outs[0] == (None, None, None)
    done = [o for o in outs if o[0] is not None] + pipe.flush_staggered(frames)
    assert len(done) == 3
    for i, (res, wav, pcm16) in enumerate(done):
        ref = seq[i][0]
        assert res.packets == ref.packets, i
        for a, b in zip(res.streams, ref.streams):
            _same_streams(a, b)
        assert torch.equal(res.n_tokens, ref.n_tokens)
        for j in range(len(res.n_tokens)):
            k = 1 + int(res.n_tokens[j])
            assert torch.equal(res.tokens[j, :k], ref.tokens[j, :k])
        if seq[i][1] is None:
            assert wav is None
            continue
        torch.testing.assert_close(wav, seq[i][1], rtol=0, atol=0)
        assert torch.equal(pcm16, seq[i][2])


def test_staggered_windows_match_seek_loop(gpu):
    """Clips of several windows (5 s, 35 s, 70 s at max_length 24: one, two and three or more
    windows of faster-whisper's seek loop) through the staggered step, batch after batch:
    every clip's seek loop — windows, seeks, <|startofprev|> prompts, segments, transcript —
    equals the drop-in's generate_segments on the same 16 kHz audio (transcriber.py:53-64),
    and the packet is the JanusPacket of that transcript. The continuation windows of
    different batches share decoder groups (the queue), so batches finish in order only
    after their last clip's last window."""
    from janus_amd.services.transcriber import generate_segments
    pipe = JanusPipeline("tiny.en", max_length=24, temperatures=(0.0,))
    specs = [[(1100 + 10 * i, 5.0), (1101 + 10 * i, 35.0), (1102 + 10 * i, 70.0)] for i in range(2)]
    batches = [_batch(gpu, sp) for sp in specs]
    frames = 8
    got = []
    for utts, pcm, offs, lengths in batches:
        r = pipe.step_staggered(pcm, offs, lengths, frames, 16, timestamp=7.0)
        if r[0] is not None:
            got.append(r)
    got += pipe.flush_staggered(frames)
    assert len(got) == 2
    for (utts, pcm, offs, lengths), (res, wav, _) in zip(batches, got):
        ref = generate_segments(pipe.whisper, [np.ascontiguousarray(u[::3]) for u in utts],
                                max_length=24, temperatures=(0.0,))
        assert [s.windows for s in ref][2] >= 3
        for b, (a, r) in enumerate(zip(res.streams, ref)):
            _same_streams(a, r)
            text = r.transcript()
            assert res.texts[b] == text
            tags = OracleProsody(48000).analyze_buffer(utts[b])[0]
            assert res.packets[b] == (opk.serialize(text, 0, tags, "auto", 7.0) if text.strip() else None)


def test_voc_dec_explicit_weights(gpu):
    """The staggered step's second vocoder context renders with the primary engine's own
    weights: a pipeline built with explicit (non-seeded, not from JANUS_VOCODER_DIR)
    vocoder weights gives bit-identical waveforms with voc_dec_utts = 2 and = 0."""
    from janus_amd import vocoder as jv
    W = jv.synthetic_weights(jv.FireflyConfig(), seed=1234)
    W = {k: (v * 1.01).astype(np.float32) if k.endswith("weight") else v for k, v in W.items()}
    out = {}
    for kv in (0, 2):
        pipe = JanusPipeline("tiny.en", max_length=12, temperatures=(0.0,), vocoder_weights=W,
                             tuning=ServingTuning(voc_dec_utts=kv))
        _, pcm, offs, lengths = _batch(gpu, [(1300 + k, 1.0 + 0.5 * k) for k in range(3)])
        r = [pipe.step_staggered(pcm, offs, lengths, 8, 16, timestamp=1.0)]
        r += pipe.flush_staggered(8)
        out[kv] = [x for x in r if x[0] is not None]
    assert len(out[0]) == len(out[2]) == 1
    torch.testing.assert_close(out[2][0][1], out[0][0][1], rtol=0, atol=0)
    assert torch.equal(out[2][0][2], out[0][0][2])


def test_pipeline_fallback_matches_seek_loop(gpu):
    """The batched pipeline with faster-whisper's fallback (temperatures 0 ... 1.0, best_of
    5: every window of the seeded synthetic model fails at T = 0) settles each utterance
    exactly as the drop-in seek loop (generate_segments) does on the same 16 kHz audio:
    same windows, tokens, segments, temperatures and sampled decodes; the overlapped
    serving step and the staggered (continuous-batching) step — whose completed windows
    that fail their gates re-decode on the whole GPU in decoder state slot 1 before their
    clips' continuation windows are queued — give the same packets, batch after batch."""
    from janus_amd.services.transcriber import TEMPERATURES, generate_segments
    pipe = JanusPipeline("tiny.en", max_length=12, temperatures=TEMPERATURES)
    utts, pcm, offs, lengths = _batch(gpu, [(500 + k, 2.0 + 3 * k) for k in range(3)])
    res = pipe.encode(pcm, offs, lengths, timestamp=5.0)
    streams = generate_segments(pipe.whisper, [np.ascontiguousarray(u[::3]) for u in utts],
                                max_length=12)
    for b, st in enumerate(streams):
        needs0, skip, avg, cr, nsp, temp, ndec, seek = res.gates[b]
        assert needs0 and ndec == 5
        _same_streams(res.streams[b], st)
        assert res.texts[b] == st.transcript()
    outs = [pipe.step_overlapped(pcm, offs, lengths, 16, 16, timestamp=5.0)]
    outs.append(pipe.flush(16))
    assert outs[1][0].packets == res.packets
    # flags, settled temperature and decode counts identical; the log-prob sums differ in
    # the last bits (the overlapped decoder runs 4 cross-attention key splits on 128 CUs)
    for g, r in zip(outs[1][0].gates, res.gates):
        assert (g[0], g[1], g[3], g[5], g[6], g[7]) == (r[0], r[1], r[3], r[5], r[6], r[7])
        assert abs(g[2] - r[2]) <= 1e-4 * abs(r[2]) and abs(g[4] - r[4]) <= 5e-3 * r[4] + 1e-9
    # the staggered step: three batches in, each settled like the seek loop
    got = []
    for _ in range(3):
        r = pipe.step_staggered(pcm, offs, lengths, 16, 16, timestamp=5.0)
        if r[0] is not None:
            got.append(r)
    got += pipe.flush_staggered(16)
    assert len(got) == 3
    for r in got:
        assert r[0].packets == res.packets
        for g, q in zip(r[0].gates, res.gates):
            assert (g[0], g[1], g[3], g[5], g[6], g[7]) == (q[0], q[1], q[3], q[5], q[6], q[7])
            assert abs(g[2] - q[2]) <= 1e-4 * abs(q[2]) and abs(g[4] - q[4]) <= 5e-3 * q[4] + 1e-9
