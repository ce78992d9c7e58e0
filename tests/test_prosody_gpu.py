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
        # numpy float32 semantics bit for bit (prosody.py:67); NaN (either sign) when empty
        if len(x):
            assert np.float32(rms[b]).view(np.uint32) == np.float32(ref_rms).view(np.uint32), \
                (b, rms[b], ref_rms)
        else:
            assert np.isnan(rms[b]) and np.isnan(ref_rms)
        voiced = [p for p in ref if p > 0]
        mf = res.mean_f0.cpu().numpy()[b]
        assert int(res.n_voiced.cpu().numpy()[b]) == len(voiced)
        if voiced:
            assert mf.view(np.uint32) == np.mean(voiced).view(np.uint32), (b, mf, np.mean(voiced))
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


def _edge_energy_hop(target_level, hop=512):
    """A hop [a, c, 0, ...] whose aubio level (sequential float sum / hop) is exactly
    target_level: a^2 just under hop*target, then c fills the last ulps."""
    from oracle.prosody import level
    E = np.float32(target_level) * np.float32(hop)           # exact (power of two)
    a = np.float32(np.sqrt(np.float64(E) * (1 - 1e-5)))
    base = np.float32(a * a)
    for c in np.float32(np.sqrt(np.float64(E - base))) * (1 + np.arange(-200, 200) * 1e-4):
        h = np.zeros(hop, np.float32)
        h[0], h[1] = a, np.float32(c)
        if level(h) == np.float32(target_level):
            return h
    raise AssertionError("no hop with that exact level")


def test_silence_gate_one_ulp(gpu):
    """aubio forces f0 = 0 when 10*log10f(level) < -50 dB. Hops whose level is the first
    non-silent float (the threshold, found with the C library's log10f) and its neighbour
    one ulp below sit inside a voiced stretch: f0 bit-identical, and the two sides of the
    gate really differ."""
    from oracle.prosody import level_db, silence_level_threshold
    thr = silence_level_threshold(-50.0)
    below = np.nextafter(thr, np.float32(0))
    above = np.nextafter(thr, np.float32(1))
    assert level_db(below) < -50.0 <= level_db(thr)
    voiced = sine(200.0, 512 * 8 / 48000, amplitude=0.3)
    parts = []
    for lv in (thr, below, above, below, thr):
        parts += [voiced, _edge_energy_hop(lv)]
    x = np.concatenate(parts + [voiced]).astype(np.float32)
    ref, _ = yin_stream(x)
    edge = [9 * k + 8 for k in range(5)]   # hop index of each edge hop
    gate = [ref[i] for i in edge]
    assert gate[1] == 0 and gate[3] == 0 and gate[0] > 0 and gate[2] > 0 and gate[4] > 0, gate
    check_batch([x], 48000, 512, gpu)


def test_yin_tolerance_straddle(gpu):
    """The early exit fires at the first tau > 4 with yin[tau-3] < tol: with tol at the
    decisive CMNDF value itself, one ulp above and one ulp below, the exit moves (or not)
    identically on the GPU and in the oracle (the comparison is strict)."""
    from oracle.prosody import yin_probe
    x = (sine(180.0, 0.2, amplitude=0.2) +
         0.05 * np.random.default_rng(5).standard_normal(9600).astype(np.float32)).astype(np.float32)
    buf = x[16 * 512 - 4096:16 * 512]               # the detector buffer at hop 15
    t, yin, _ = yin_probe(buf, 0.8)
    assert t > 0
    v = yin[t - 3]                                  # the value that decided the exit
    for tol in (v, np.nextafter(v, np.float32(2)), np.nextafter(v, np.float32(0))):
        ref, _ = yin_stream(x, tol=float(tol))
        lengths = [len(x)]
        offs = torch.tensor([0, len(x)], dtype=torch.int64, device=gpu)
        pcm = torch.from_numpy(np.concatenate([x, np.zeros(1, np.float32)])).to(gpu)
        res = prosody_launch(pcm, offs, lengths, 48000, 512, tolerance=float(tol))
        torch.cuda.synchronize()
        assert np.array_equal(res.f0.cpu().numpy().view(np.uint32), ref.view(np.uint32)), tol


def test_yin_near_tolerance_at_0_8(gpu):
    """At the reference's tolerance 0.8: the noise level of a noisy 150 Hz buffer is
    bisected until the smallest CMNDF local minimum (the value that decides whether the
    early exit fires at all) is one ulp below 0.8 in one buffer and exactly 0.8f in the
    next — exit vs argmin path, bit-identical on the GPU."""
    from oracle.prosody import yin_probe
    rng = np.random.default_rng(11)
    s = sine(150.0, 4096 / 48000, amplitude=0.3)
    n = rng.standard_normal(4096).astype(np.float32)

    def crit(alpha):
        buf = (s + np.float32(alpha) * n).astype(np.float32)
        _, yin, _ = yin_probe(buf, -1.0)            # full CMNDF (no exit)
        p = np.arange(2, 2047)
        return buf, np.float32(yin[p][yin[p] < yin[p + 1]].min())

    lo, hi = 0.3, 10.0
    for _ in range(64):
        mid = 0.5 * (lo + hi)
        if crit(mid)[1] < np.float32(0.8):
            lo = mid
        else:
            hi = mid
    b_lo, v_lo = crit(lo)
    b_hi, v_hi = crit(hi)
    assert v_lo == np.nextafter(np.float32(0.8), np.float32(0)) and v_hi == np.float32(0.8), (v_lo, v_hi)
    assert yin_probe(b_lo, 0.8)[0] > 0 and yin_probe(b_hi, 0.8)[0] == -1   # exit vs no exit
    check_batch([b_lo.copy(), b_hi.copy()], 48000, 512, gpu)


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


# ---- numpy-exact energy and voiced-f0 means at the tag edges ---------

def _rms_np(x):
    return np.sqrt(np.mean(x ** 2))


def _buffers_at(target, n, seed):
    """Buffers whose numpy rms is exactly prev(target), target and next(target) (float32):
    one random buffer scaled near the target, then its largest sample a set by bisection
    over the float32 bit patterns (numpy's rms is monotone in a: every float op on the way
    is) to the smallest a whose rms reaches each wanted value."""
    for s in range(seed, seed + 1000, 100):   # large sums can step over an rms value
        out = _try_buffers_at(target, n, s)
        if out is not None:
            return out
    raise AssertionError("no buffer reaches the wanted rms values")


def _try_buffers_at(target, n, seed):
    t = np.float32(target)
    x = np.random.default_rng(seed).standard_normal(n).astype(np.float32)
    y = (np.abs(x) * np.float32(float(target) / float(_rms_np(x)))).astype(np.float32)
    i = int(np.argmax(y))
    out = []
    for want in (np.nextafter(t, np.float32(0)), t, np.nextafter(t, np.float32(np.inf))):
        lo, hi = 0, int(np.float32(4.0 * float(y[i]) + 1.0).view(np.uint32))
        while hi - lo > 1:
            mid = (lo + hi) // 2
            y[i] = np.array(mid, np.uint32).view(np.float32)
            if _rms_np(y) >= want:
                hi = mid
            else:
                lo = mid
        y[i] = np.array(hi, np.uint32).view(np.float32)
        if _rms_np(y) != want:
            return None
        out.append((want, y.copy()))
    return out


@pytest.mark.parametrize("target", [0.05, 0.15])
def test_energy_tag_edges_bit_exact(gpu, target):
    """Buffers whose numpy rms is 0.05f / 0.15f and one ulp either side (lengths spanning
    several 8192-sample numpy buffers plus a ragged tail): GPU rms bit-identical, tags equal
    to the reference's (Quiet|Normal / Normal|Loud flip exactly where numpy's does)."""
    cases = _buffers_at(target, 3 * 8192 + 77, 7) + _buffers_at(target, 150001, 8)
    bufs = [y for _, y in cases]
    res, _ = run_batch(bufs, 48000, 512, gpu)
    rms = res.rms.cpu().numpy()
    tags = res.tags()
    for b, (r, y) in enumerate(cases):
        assert rms[b].view(np.uint32) == r.view(np.uint32), (b, rms[b], r)
        assert tags[b]['energy'] == energy_tag(r)
    assert {energy_tag(r) for r, _ in cases} == ({'Quiet', 'Normal'} if target == 0.05 else {'Normal', 'Loud'})


def test_energy_ragged_offsets_bit_exact(gpu):
    """64 utterances at arbitrary (unaligned) offsets and lengths 0 .. 3 numpy buffers: rms
    bit-identical to numpy (the 16-byte and the scalar leaf paths)."""
    rng = np.random.default_rng(21)
    lengths = [0, 1, 7, 8, 127, 128, 129, 8191, 8192, 8193] + [int(v) for v in rng.integers(1, 30000, 54)]
    bufs = [(rng.standard_normal(n) * rng.uniform(0.01, 1)).astype(np.float32) for n in lengths]
    res, _ = run_batch(bufs, 48000, 512, gpu)
    rms = res.rms.cpu().numpy()
    for b, x in enumerate(bufs):
        with np.errstate(all="ignore"):
            ref = _rms_np(x)
        if len(x) == 0:
            assert np.isnan(rms[b])
            continue
        assert rms[b].view(np.uint32) == ref.view(np.uint32), (b, len(x), rms[b], ref)


def _voiced_mean_gpu(lists, gpu):
    from janus_amd import _native as nat
    offs = np.concatenate([[0], np.cumsum([len(v) for v in lists])]).astype(np.int64)
    vals = torch.from_numpy(np.concatenate(lists + [np.zeros(1, np.float32)]).astype(np.float32)).to(gpu)
    o = torch.from_numpy(offs).to(gpu)
    mean = torch.empty(len(lists), dtype=torch.float32, device=gpu)
    cnt = torch.empty(len(lists), dtype=torch.int32, device=gpu)
    nat.call("janus_np_voiced_mean_f32", vals.data_ptr(), o.data_ptr(), len(lists), mean.data_ptr(),
             cnt.data_ptr(), nat.stream_ptr(gpu))
    torch.cuda.synchronize()
    return mean.cpu().numpy(), cnt.cpu().numpy()


def _f0_lists_at(target, n, seed):
    """f0 lists (n a power of two, so the mean is the sum scaled exactly) whose numpy mean of
    the positive values is prev(target), target, next(target); unvoiced zeros interleaved."""
    rng = np.random.default_rng(seed)
    base = rng.uniform(0.5 * target, 1.5 * target, n).astype(np.float32)   # all voiced (> 0)
    base = (base - base.mean() + np.float32(target)).astype(np.float32)
    t = np.float32(target)
    want = {np.nextafter(t, np.float32(0)): None, t: None, np.nextafter(t, np.float32(np.inf)): None}
    last = float(base[-1])
    step = float(np.spacing(np.float32(target))) * n / 64
    for k in range(-20000, 20000):
        v = base.copy()
        v[-1] = np.float32(last + k * step)
        m = np.mean(v)
        if m in want and want[m] is None:
            want[m] = v
        if all(x is not None for x in want.values()):
            break
    assert all(x is not None for x in want.values())
    out = []
    for m, v in want.items():
        z = np.zeros(len(v) + len(v) // 3, np.float32)
        pos = np.sort(rng.choice(len(z), len(v), replace=False))
        z[pos] = v
        out.append((m, z))
    return out


@pytest.mark.parametrize("target", [120.0, 200.0])
def test_pitch_tag_edges_bit_exact(gpu, target):
    """Voiced-f0 means at 120f / 200f and one ulp either side (np.mean over the positive
    values in hop order, prosody.py:86-90), with 256 and 16384 voiced values (the latter
    spans two numpy buffers): GPU mean and count bit-identical, pitch tag flips exactly
    where the reference's does."""
    cases = _f0_lists_at(target, 256, 3) + _f0_lists_at(target, 16384, 4)
    mean, cnt = _voiced_mean_gpu([z for _, z in cases], gpu)
    for b, (m, z) in enumerate(cases):
        voiced = [p for p in z if p > 0]
        assert cnt[b] == len(voiced)
        assert mean[b].view(np.uint32) == m.view(np.uint32) == np.mean(voiced).view(np.uint32)
        from janus_amd.services.prosody import pitch_tag as gpu_tag
        assert gpu_tag(float(mean[b]), int(cnt[b])) == pitch_tag(voiced)
    tags = {pitch_tag([m]) for m, _ in cases}
    assert tags == ({'Deep', 'Normal'} if target == 120.0 else {'Normal', 'High'})


def test_voiced_mean_random_bit_exact(gpu):
    rng = np.random.default_rng(9)
    lists = [np.zeros(0, np.float32), np.zeros(10, np.float32)]
    for n in (1, 7, 8, 9, 128, 129, 1000, 2813, 8192, 8193, 9000, 20000):
        v = rng.uniform(50, 1500, n).astype(np.float32)
        v[rng.random(n) < 0.3] = 0.0
        lists.append(v)
    mean, cnt = _voiced_mean_gpu(lists, gpu)
    for b, v in enumerate(lists):
        pos = v[v > 0]
        assert cnt[b] == len(pos)
        if len(pos):
            assert mean[b].view(np.uint32) == np.mean(pos).view(np.uint32), (b, len(v))
        else:
            assert mean[b] == 0.0
