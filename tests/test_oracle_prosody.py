"""Oracle pinning for the prosody path (CPU): the sequential aubio-YIN restatement
reproduces the reference's own known-answer tests
(backend/tests/test_input_processing.py:436-505)."""
import numpy as np

from janus_amd.workload import sine, synth_speech
from oracle.prosody import (NP_BUFSIZE, PW_DEPTH, OracleProsody, np_mean_f32, np_sum_f32,
                            pairwise_sum_f32, pw_slot, yin_stream)


def test_kat_energy_quiet():              # test_input_processing.py:461-468
    r, _, _ = OracleProsody(48000).analyze_buffer(sine(amplitude=0.02, duration=0.5))
    assert r['energy'] == 'Quiet'


def test_kat_energy_ranges():             # :470-478
    ex = OracleProsody(48000)
    assert ex.analyze_buffer(sine(amplitude=0.1, duration=0.5))[0]['energy'] in ('Quiet', 'Normal')
    assert ex.analyze_buffer(sine(amplitude=0.5, duration=0.5))[0]['energy'] in ('Normal', 'Loud')


def test_kat_440hz_is_high():             # :480-490
    r, f0, _ = OracleProsody(48000).analyze_buffer(sine(440.0, 0.5, amplitude=0.3))
    assert r['pitch'] == 'High'
    voiced = f0[f0 > 0]
    assert len(voiced) > 0 and abs(np.median(voiced) - 440.0) < 2.0


def test_kat_list_input():                # :492-505
    ex = OracleProsody(48000)
    r, _, _ = ex.analyze_buffer([sine(220.0, 0.25, amplitude=0.2), sine(220.0, 0.25, amplitude=0.2)])
    assert set(r) == {'energy', 'pitch'} and list(r) == ['energy', 'pitch']


def test_keys_order_and_values():         # :447-459
    r, _, _ = OracleProsody(48000).analyze_buffer(sine(440.0, 0.5, amplitude=0.3))
    assert list(r) == ['energy', 'pitch']
    assert r['energy'] in ('Quiet', 'Normal', 'Loud') and r['pitch'] in ('Deep', 'Normal', 'High')


def test_silence_gives_zero_pitch():
    f0, _ = yin_stream(np.zeros(4096, np.float32))
    assert np.all(f0 == 0)


def test_pitch_tracks_sine_frequencies():
    for f in (110.0, 165.0, 330.0):
        f0, _ = yin_stream(sine(f, 0.5, amplitude=0.3))
        v = f0[f0 > 0][8:]  # after the 4096-sample buffer has filled
        assert abs(np.median(v) - f) < 0.01 * f


def test_state_carries_across_calls():
    x = sine(200.0, 0.5, amplitude=0.3)
    whole, st_whole = yin_stream(x)
    a, st = yin_stream(x[:512 * 20])
    b, st2 = yin_stream(x[512 * 20:], state=st)
    assert np.array_equal(np.concatenate([a, b]), whole)
    assert np.array_equal(st2, st_whole)


def test_synthetic_speech_classes():
    ex = OracleProsody(48000)
    # The workload's F0 classes sit away from the 120/200 Hz edges; the tag itself is the
    # mean of every positive hop, which aubio also fills with onset outliers (period < 1),
    # so the robust check is the median of the voiced hops.
    for f0c in (95.0, 160.0, 260.0):
        x = synth_speech(7, 2.0, f0=f0c, rms=0.10)
        r, f0, rms = OracleProsody(48000).analyze_buffer(x)
        assert r['energy'] == 'Normal' and abs(rms - 0.10) < 1e-3
        assert abs(np.median(f0[f0 > 0]) - f0c) < 0.05 * f0c


# ---- numpy float32 reductions (prosody.py:67 rms, :90 mean of voiced f0) -----------------

def test_np_sum_restatement_matches_numpy():
    """The reduction the GPU reproduces — 8192-element buffers, pairwise inside, sequential
    across — equals numpy's own np.sum / np.mean on float32 bit for bit (sizes around the
    leaf, split and buffer boundaries and up to a 30 s 48 kHz buffer)."""
    rng = np.random.default_rng(0)
    sizes = list(range(0, 300)) + [1000, 1023, 4096, 8191, 8192, 8193, 8199, 16384, 16385,
                                   24575, 100000, 1440000]
    sizes += [int(v) for v in rng.integers(1, 400000, 40)]
    for n in sizes:
        x = (rng.standard_normal(n) * rng.uniform(0.01, 3.0)).astype(np.float32)
        sq = x ** 2
        assert np_sum_f32(sq).view(np.uint32) == np.sum(sq).view(np.uint32), n
        if n:
            with np.errstate(all="ignore"):
                assert np_mean_f32(sq).view(np.uint32) == np.mean(sq).view(np.uint32), n
    # the mean of a list of np.float32 scalars (pitch_values, prosody.py:87-90)
    vals = [np.float32(v) for v in rng.uniform(80, 400, 3000)]
    assert np_mean_f32(np.array(vals, np.float32)) == np.mean(vals)


def test_np_sum_is_not_plain_pairwise():
    """Sanity: the 8192 buffering matters (a whole-array pairwise tree differs)."""
    rng = np.random.default_rng(1)
    diff = 0
    for _ in range(20):
        sq = (rng.standard_normal(100000).astype(np.float32)) ** 2
        diff += pairwise_sum_f32(sq) != np.sum(sq)
    assert diff > 0


def test_gpu_slot_map_covers_every_buffer():
    """The GPU's 128-slot map (zero slots padded into a perfect tree) reaches every leaf of
    every buffer length <= 8192 within 7 levels and reproduces pairwise_sum exactly."""
    rng = np.random.default_rng(2)
    for m in range(0, NP_BUFSIZE + 1):
        slots = [pw_slot(m, t) for t in range(1 << PW_DEPTH)]   # asserts depth <= 7
        if m == NP_BUFSIZE:   # the GPU's full-buffer fast path: slot 2i owns (128 i, 128)
            assert slots == [(128 * (t // 2), 128) if t % 2 == 0 else None for t in range(128)]
        got = [s for s in slots if s is not None]
        assert sum(ln for _, ln in got) == m and all(ln <= 128 for _, ln in got)
        if m % 97 == 0 or m in (8190, 8191, 8192):
            a = (rng.standard_normal(m).astype(np.float32)) ** 2
            vals = [np.float32(0)] * (1 << PW_DEPTH)
            from oracle.prosody import _pw_leaf
            for t, s in enumerate(slots):
                if s is not None:
                    vals[t] = _pw_leaf(a[s[0]:s[0] + s[1]])
            while len(vals) > 1:
                vals = [np.float32(vals[2 * i] + vals[2 * i + 1]) for i in range(len(vals) // 2)]
            assert vals[0] == pairwise_sum_f32(a), m
