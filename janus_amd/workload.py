"""Seeded synthetic speech — inputs for tests and the bench.

No datasets or recordings are reachable, so the workload is source-filter
"speech": a glottal pulse train with ±3 % vibrato at an F0 drawn from
{95, 160, 260} Hz (away from the 120/200 Hz pitch-bucket edges of prosody.py:92-97),
three formant resonators (500/1500/2500 Hz), 4 Hz syllabic amplitude modulation,
10 % noise bursts and 150-300 ms pauses, RMS-scaled to {0.03, 0.10, 0.25} (away from
the 0.05/0.15 energy edges of prosody.py:69-74). Generated in float64 at 48 kHz,
quantised to int16 and divided by 32768 exactly as audio_io.py:125-126 does; the
Whisper input is the reference's plain ``[::3]`` decimation (transcriber.py:51).
Seed = 1000·config + utterance index.
"""
import numpy as np
from scipy.signal import lfilter

F0_CLASSES = (95.0, 160.0, 260.0)
RMS_CLASSES = (0.03, 0.10, 0.25)
FORMANTS = ((500.0, 200.0), (1500.0, 300.0), (2500.0, 400.0))


def _resonator(freq, bw, sr):
    r = np.exp(-np.pi * bw / sr)
    theta = 2 * np.pi * freq / sr
    a = [1.0, -2 * r * np.cos(theta), r * r]
    b = [1.0 - r]
    return b, a


def synth_speech(seed: int, seconds: float = 30.0, sr: int = 48000, f0: float = None,
                 rms: float = None) -> np.ndarray:
    """float32 PCM in [-1, 1) on the int16 grid, length round(seconds*sr)."""
    rng = np.random.default_rng(seed)
    n = int(round(seconds * sr))
    if n == 0:
        return np.zeros(0, np.float32)
    f0 = float(rng.choice(F0_CLASSES)) if f0 is None else float(f0)
    rms = float(rng.choice(RMS_CLASSES)) if rms is None else float(rms)
    t = np.arange(n) / sr
    vib = 1.0 + 0.03 * np.sin(2 * np.pi * 5.5 * t + rng.uniform(0, 2 * np.pi))
    phase = np.cumsum(f0 * vib) / sr
    frac = phase - np.floor(phase)
    # Rosenberg-like glottal pulse: open phase 60 % of the period.
    op = 0.6
    pulse = np.where(frac < op, 0.5 * (1 - np.cos(np.pi * frac / op)), 0.0)
    src = pulse - pulse.mean()
    x = src.copy()
    for k, (fc, bw) in enumerate(FORMANTS):
        b, a = _resonator(fc * rng.uniform(0.95, 1.05), bw, sr)
        y = lfilter(b, a, src)
        x += (0.5 / (k + 1)) * y * (np.std(src) / (np.std(y) + 1e-12))
    am = 0.55 + 0.45 * np.sin(2 * np.pi * 4.0 * t + rng.uniform(0, 2 * np.pi))
    x *= am
    # 10 % noise bursts (fricatives), 30-80 ms each.
    noise = np.zeros(n)
    pos = 0
    while pos < n:
        pos += int(rng.uniform(0.3, 0.7) * sr)
        ln = int(rng.uniform(0.03, 0.08) * sr)
        if pos < n:
            noise[pos:pos + ln] = rng.standard_normal(min(ln, n - pos))
    x += noise * (np.std(x) + 1e-12) * 0.15
    # 150-300 ms pauses every ~1.5 s.
    pos = int(rng.uniform(0.5, 1.5) * sr)
    while pos < n:
        ln = int(rng.uniform(0.15, 0.3) * sr)
        x[pos:pos + ln] = 0.0
        pos += ln + int(rng.uniform(1.0, 2.0) * sr)
    cur = np.sqrt(np.mean(x * x)) + 1e-20
    x *= rms / cur
    q = np.clip(np.round(x * 32768.0), -32768, 32767).astype(np.int16)
    return (q.astype(np.float32) / 32768.0).astype(np.float32)


def utterance_batch(config: int, count: int, seconds: float = 30.0, sr: int = 48000):
    """List of `count` utterances with seeds 1000*config + idx."""
    return [synth_speech(1000 * config + i, seconds, sr) for i in range(count)]


def channel_audio(channel: int, n_samples: int, sr: int = 48000) -> np.ndarray:
    """One capture channel of BASELINE config 5 (48 kHz): phrases of 1.5-6 s separated by
    0.6-2 s of silence, the first starting within 1 s. Seeded per GLOBAL channel index
    (5000 + channel), so a rank generates only the channels it owns and every world size
    sees the same channels."""
    rng = np.random.default_rng(5000 + channel)
    out = np.zeros(n_samples, np.float32)
    t = int(rng.integers(0, sr))
    k = 0
    while t < n_samples:
        ph = synth_speech(5000 + 97 * channel + k, float(rng.uniform(1.5, 6.0)), sr)
        n = min(len(ph), n_samples - t)
        out[t:t + n] = ph[:n]
        t += n + int(rng.uniform(0.6, 2.0) * sr)
        k += 1
    return out


def sine(frequency=440.0, duration=1.0, sample_rate=48000, amplitude=0.5) -> np.ndarray:
    """Same construction as the reference's generate_sine_wave
    (backend/tests/test_input_processing.py:30-45)."""
    t = np.linspace(0, duration, int(sample_rate * duration), dtype=np.float32)
    return amplitude * np.sin(2 * np.pi * frequency * t, dtype=np.float32)
