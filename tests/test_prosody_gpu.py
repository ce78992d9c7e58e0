"""GPU parity for the prosody path: janus_prosody_analyze vs the sequential aubio-YIN
oracle — per-hop f0 bit-identical, state bit-identical, tags identical.
Mirrors backend/tests/test_input_processing.py:436-505 on the drop-in class."""
import numpy as np
import pytest
import torch

from janus_amd.services.prosody import ProsodyExtractor, prosody_launch
from janus_amd.workload import sine, synth_speech
from oracle.prosody import OracleProsody, energy_tag, pitch_tag, yin_stream

pytestmark = pytest.mark.gpu


def run_batch(bufs, sr, hop, dev, states=None):
    lengths = [len(b) for b in bufs]
    offs = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    pcm = torch.from_numpy(np.concatenate(bufs + [np.zeros(1, np.float32)]).astype(np.float32)).to(dev)
    so = torch.from_numpy(offs).to(dev)
    st_in = None if states is None else torch.from_numpy(np.stack(states)).to(dev).reshape(-1)
    st_out = torch.empty(len(bufs) * 4096, dtype=torch.float32, device=dev)
    res = prosody_launch(pcm, so, lengths, sr, hop, state_in=st_in, state_out=st_out)
    torch.cuda.synchronize()
    return res, st_out.cpu().numpy().reshape(len(bufs), 4096)


def check_batch(bufs, sr, hop, dev, states=None):
    res, st = run_batch(bufs, sr, hop, dev, states)
    f0 = res.f0.cpu().numpy()
    rms = res.rms.cpu().numpy()
    tags = res.tags()
    for b, x in enumerate(bufs):
        ref, ref_st = yin_stream(x, sr, hop, state=None if states is None else states[b])
        got = f0[res.hop_off[b]:res.hop_off[b + 1]]
        assert got.shape == ref.shape
        bad = np.nonzero(got.view(np.uint32) != ref.view(np.uint32))[0]
        assert bad.size == 0, f"utt {b}: {bad.size} hops differ, first {bad[:5]}: {got[bad[:5]]} vs {ref[bad[:5]]}"
        assert np.array_equal(st[b].view(np.uint32), ref_st.view(np.uint32))
        with np.errstate(all="ignore"):
            ref_rms = np.sqrt(np.mean(x.astype(np.float32) ** 2))
        if len(x):
            assert abs(rms[b] - ref_rms) <= 1e-6 * max(ref_rms, 1e-6)
        else:
            assert np.isnan(rms[b])
        voiced = [p for p in ref if p > 0]
        assert tags[b] == {'energy': energy_tag(ref_rms), 'pitch': pitch_tag(voiced)}


def test_sines_bit_exact(gpu):
    bufs = [sine(440.0, 0.5, amplitude=0.3), sine(110.0, 0.4, amplitude=0.02),
            sine(220.0, 0.25, amplitude=0.5), sine(1000.0, 0.3, amplitude=0.1)]
    check_batch(bufs, 48000, 512, gpu)


def test_speech_ragged_bit_exact(gpu):
    rng = np.random.default_rng(3)
    bufs = [synth_speech(100 + k, 1.0 + 0.37 * k) for k in range(3)]
    bufs += [np.zeros(0, np.float32), rng.standard_normal(100).astype(np.float32) * 0.1,
             np.zeros(5000, np.float32), (rng.standard_normal(7777) * 0.2).astype(np.float32)]
    check_batch(bufs, 48000, 512, gpu)


@pytest.mark.parametrize("sr,hop", [(16000, 512), (48000, 256), (44100, 1024)])
def test_other_rates_and_hops(gpu, sr, hop):
    bufs = [synth_speech(200, 0.8, sr=sr), sine(300.0, 0.6, sample_rate=sr, amplitude=0.2)]
    check_batch(bufs, sr, hop, gpu)


def test_state_carry(gpu):
    x = synth_speech(300, 1.5)
    cut = 512 * 37 + 100
    _, st = run_batch([x[:cut]], 48000, 512, gpu)
    check_batch([x[cut:]], 48000, 512, gpu, states=[st[0]])


def test_dropin_known_answers(gpu):
    ex = ProsodyExtractor(sample_rate=48000, hop_size=512)
    assert ex.sample_rate == 48000 and ex.hop_size == 512 and ex.pitch_detector is not None
    assert ex.analyze_buffer(sine(amplitude=0.02, duration=0.5))['energy'] == 'Quiet'
    assert ex.analyze_buffer(sine(amplitude=0.1, duration=0.5))['energy'] in ('Quiet', 'Normal')
    assert ex.analyze_buffer(sine(amplitude=0.5, duration=0.5))['energy'] in ('Normal', 'Loud')
    r = ProsodyExtractor(48000).analyze_buffer(sine(440.0, 0.5, amplitude=0.3))
    assert r == {'energy': 'Loud', 'pitch': 'High'} and list(r) == ['energy', 'pitch']  # rms 0.212
    r = ex.analyze_buffer([sine(220.0, 0.25, amplitude=0.2), sine(220.0, 0.25, amplitude=0.2)])
    assert set(r) == {'energy', 'pitch'}


def test_dropin_stateful_matches_oracle(gpu):
    ex, orc = ProsodyExtractor(48000), OracleProsody(48000)
    for k in range(3):
        x = synth_speech(400 + k, 0.7)
        assert ex.analyze_buffer(x) == orc.analyze_buffer(x)[0]
    assert np.array_equal(ex.pitch_detector.state.cpu().numpy(), orc.state)


def test_per_hop_call_api(gpu):
    ex = ProsodyExtractor(48000)
    x = sine(330.0, 0.3, amplitude=0.3)
    ref, _ = yin_stream(x)
    got = [ex.pitch_detector(np.pad(x[i:i + 512], (0, max(0, i + 512 - len(x)))))[0]
           for i in range(0, len(x), 512)]
    assert np.array_equal(np.array(got, np.float32), ref)


@pytest.mark.parametrize("max_blocks", [1, 7, 256])
def test_grid_cap_identical(gpu, max_blocks):
    """janus_prosody_analyze_ex with a capped grid (the pipeline's prosody-beside-decoder
    launch) gives per-hop f0 bit-identical to one block per hop."""
    bufs = [synth_speech(900 + k, 0.7 + 0.3 * k) for k in range(4)]
    lengths = [len(b) for b in bufs]
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)).to(gpu)
    pcm = torch.from_numpy(np.concatenate(bufs + [np.zeros(1, np.float32)])).to(gpu)
    a = prosody_launch(pcm, offs, lengths, 48000, 512)
    b = prosody_launch(pcm, offs, lengths, 48000, 512, max_blocks=max_blocks)
    torch.cuda.synchronize()
    assert np.array_equal(a.f0.cpu().numpy().view(np.uint32), b.f0.cpu().numpy().view(np.uint32))
    assert a.tags() == b.tags()
