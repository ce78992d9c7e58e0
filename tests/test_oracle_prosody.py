"""Oracle pinning for the prosody path (CPU): the sequential aubio-YIN restatement
reproduces the reference's own known-answer tests
(backend/tests/test_input_processing.py:436-505)."""
import numpy as np

from janus_amd.workload import sine, synth_speech
from oracle.prosody import OracleProsody, yin_stream


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
