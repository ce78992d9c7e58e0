"""ORACLE — test infrastructure only (see oracle/__init__.py).

CPU restatement of ``ProsodyExtractor`` (backend/services/prosody.py:11-104):
energy from numpy float32 RMS (:67-74), pitch from the sequential aubio-YIN
restatement in oracle/yin_oracle.c (:32-34, :78-87), mean of voiced pitches and
bucketing (:89-99), result dict in ``energy, pitch`` order (:101-104).

Pinned by the reference's known-answer tests (tests/test_oracle.py):
test_input_processing.py:461-468 (0.02 amplitude -> 'Quiet'), :470-478 (ranges),
:480-490 (440 Hz sine -> 'High'), :492-505 (list input).
"""
import ctypes
import os

import numpy as np

from . import BUILD_DIR, build

YIN_BUF = 4096
DEFAULT_SILENCE_DB = -50.0   # aubio src/pitch/pitch.c DEFAULT_PITCH_SILENCE
DEFAULT_TOLERANCE = 0.8      # prosody.py:34

_lib = None


def _load():
    global _lib
    if _lib is None:
        path = os.path.join(BUILD_DIR, "libjanus_oracle.so")
        if not os.path.exists(path):
            build()
        lib = ctypes.CDLL(path)
        lib.yin_oracle_stream.argtypes = [
            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_float,
            ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
        lib.yin_oracle_stream.restype = None
        lib.yin_oracle_level.argtypes = [ctypes.c_void_p, ctypes.c_uint]
        lib.yin_oracle_level.restype = ctypes.c_float
        lib.yin_oracle_db.argtypes = [ctypes.c_float]
        lib.yin_oracle_db.restype = ctypes.c_float
        lib.yin_oracle_probe.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
        lib.yin_oracle_probe.restype = ctypes.c_int
        _lib = lib
    return _lib


def level(hop_samples) -> np.float32:
    """aubio_level_lin of one hop (sequential float sum / n)."""
    x = np.ascontiguousarray(hop_samples, np.float32)
    return np.float32(_load().yin_oracle_level(x.ctypes.data, len(x)))


def level_db(lv) -> np.float32:
    """The dB value aubio_silence_detection compares with the threshold."""
    return np.float32(_load().yin_oracle_db(float(lv)))


def silence_level_threshold(silence_db=DEFAULT_SILENCE_DB) -> np.float32:
    """Smallest float level that is NOT silent under level_db (bisection over bits)."""
    lo, hi = 0, 0x7F800000
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if level_db(np.array(mid, np.uint32).view(np.float32)) < silence_db:
            lo = mid
        else:
            hi = mid
    return np.array(hi, np.uint32).view(np.float32)


def yin_probe(buf4096, tol=DEFAULT_TOLERANCE):
    """(exit tau or -1, CMNDF up to the exit, period) of one detector buffer."""
    b = np.ascontiguousarray(buf4096, np.float32)
    assert b.shape == (YIN_BUF,)
    yin = np.zeros(YIN_BUF // 2, np.float32)
    per = ctypes.c_float()
    t = _load().yin_oracle_probe(b.ctypes.data, tol, yin.ctypes.data, ctypes.addressof(per))
    return t, yin, per.value


def yin_stream(x, sample_rate=48000, hop=512, tol=DEFAULT_TOLERANCE,
               silence_db=DEFAULT_SILENCE_DB, state=None):
    """Per-hop f0 (Hz) of a stream, aubio semantics. Returns (f0[nhops], new_state)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    st = np.zeros(YIN_BUF, np.float32) if state is None else np.array(state, np.float32, copy=True)
    nh = (len(x) + hop - 1) // hop
    f0 = np.zeros(max(nh, 0), np.float32)
    _load().yin_oracle_stream(x.ctypes.data, len(x), sample_rate, hop, tol, silence_db,
                              st.ctypes.data, f0.ctypes.data)
    return f0, st


NP_BUFSIZE = 8192   # numpy's reduction buffer (NPY_BUFSIZE)
PW_BLOCKSIZE = 128  # numpy pairwise_sum leaf size
PW_DEPTH = 7        # leaves of a buffer <= 8192 lie at depth <= 7 (128 slots on the GPU)


def _pw_leaf(a):
    """numpy/_core/src/umath/loops_utils.h.src pairwise_sum for n <= 128 (float32)."""
    n = len(a)
    f = np.float32
    if n < 8:
        r = f(0)
        for v in a:
            r = f(r + v)
        return r
    r = [f(v) for v in a[:8]]
    i = 8
    while i < n - (n % 8):
        for j in range(8):
            r[j] = f(r[j] + a[i + j])
        i += 8
    res = f(f(f(r[0] + r[1]) + f(r[2] + r[3])) + f(f(r[4] + r[5]) + f(r[6] + r[7])))
    for k in range(i, n):
        res = f(res + a[k])
    return res


def pairwise_sum_f32(a):
    """numpy's float32 pairwise_sum over one buffer: split at n/2 rounded down to a
    multiple of 8 until a block is <= 128."""
    n = len(a)
    if n <= PW_BLOCKSIZE:
        return _pw_leaf(a)
    n2 = n // 2
    n2 -= n2 % 8
    return np.float32(pairwise_sum_f32(a[:n2]) + pairwise_sum_f32(a[n2:]))


def np_sum_f32(a):
    """np.add.reduce of a contiguous float32 array: the reduction iterator feeds buffers of
    8192 elements, each pairwise-summed, accumulated in order into the identity 0.0f."""
    a = np.ascontiguousarray(a, np.float32)
    out = np.float32(0)
    for i in range(0, len(a), NP_BUFSIZE):
        out = np.float32(out + pairwise_sum_f32(a[i:i + NP_BUFSIZE]))
    return out


def np_mean_f32(a):
    """np.mean of a float32 array: float32 sum, float64 divide by the np.intp count
    (numpy/_core/_methods.py _mean), cast back to float32."""
    return np.float32(np.float64(np_sum_f32(a)) / np.float64(len(a)))


def pw_slot(m, t):
    """The GPU's slot map (csrc/prosody.hip pw_slot): (offset, length) of the leaf slot t
    of a buffer of m <= 8192 owns, or None for a zero slot."""
    off, ln = 0, m
    for lvl in range(PW_DEPTH):
        if ln <= PW_BLOCKSIZE:
            return (off, ln) if t & ((1 << (PW_DEPTH - lvl)) - 1) == 0 else None
        n2 = ln // 2
        n2 -= n2 % 8
        if (t >> (PW_DEPTH - 1 - lvl)) & 1:
            off, ln = off + n2, ln - n2
        else:
            ln = n2
    assert ln <= PW_BLOCKSIZE, (m, t, ln)
    return off, ln


def energy_tag(rms) -> str:
    """prosody.py:69-74 (NaN from an empty buffer compares False -> 'Loud')."""
    if rms < 0.05:
        return 'Quiet'
    elif rms < 0.15:
        return 'Normal'
    return 'Loud'


def pitch_tag(voiced) -> str:
    """prosody.py:89-99."""
    if len(voiced) > 0:
        avg = np.mean(voiced)
        if avg < 120:
            return 'Deep'
        elif avg < 200:
            return 'Normal'
        return 'High'
    return 'Normal'


class OracleProsody:
    """Stateful mirror of ProsodyExtractor on the CPU (one aubio buffer per object)."""

    def __init__(self, sample_rate: int = 48000, hop_size: int = 512):
        self.sample_rate = sample_rate
        self.hop_size = hop_size
        self.state = np.zeros(YIN_BUF, np.float32)

    def analyze_buffer(self, audio_buffer):
        if isinstance(audio_buffer, list):
            audio_buffer = np.concatenate(audio_buffer)
        if not isinstance(audio_buffer, np.ndarray):
            audio_buffer = np.array(audio_buffer, dtype=np.float32)
        if audio_buffer.dtype != np.float32:
            audio_buffer = audio_buffer.astype(np.float32)
        with np.errstate(all='ignore'):
            rms = np.sqrt(np.mean(audio_buffer ** 2))
        f0, self.state = yin_stream(audio_buffer, self.sample_rate, self.hop_size,
                                    state=self.state)
        voiced = [p for p in f0 if p > 0.0]
        return {'energy': energy_tag(rms), 'pitch': pitch_tag(voiced)}, f0, rms
