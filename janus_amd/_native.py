"""Loader for libjanus_hip.so, the gfx950 HIP library behind include/janus.h.

torch is imported first so that libjanus_hip.so binds to the same HIP runtime
(libamdhip64.so.7) torch already loaded; device pointers from torch tensors are then
valid in both. There is no fallback: if the library is missing or fails to load,
every janus_amd entry point raises.
"""
import ctypes

import numpy as np
import os

import torch  # noqa: F401  (must precede the dlopen below)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libjanus_hip.so")
# A/B experiments only: JANUS_LIB names an alternative in-tree build (e.g. libjanus_hip_nt.so)
if os.environ.get("JANUS_LIB"):
    LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), os.path.basename(os.environ["JANUS_LIB"]))


class JanusNativeError(RuntimeError):
    """A libjanus_hip.so entry point returned a non-zero status."""


class janus_value(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("i", ctypes.c_int64), ("f", ctypes.c_double),
                ("s", ctypes.c_char_p), ("len", ctypes.c_size_t)]


class janus_packet(ctypes.Structure):
    _fields_ = [("text", ctypes.c_char_p), ("text_len", ctypes.c_size_t),
                ("mode", ctypes.c_int64), ("n_prosody", ctypes.c_int32),
                ("prosody_keys", ctypes.POINTER(janus_value)),
                ("prosody_vals", ctypes.POINTER(janus_value)),
                ("override_emotion", ctypes.c_char_p), ("override_len", ctypes.c_size_t),
                ("timestamp", janus_value)]


class janus_mp_node(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("i", ctypes.c_int64), ("f", ctypes.c_double),
                ("offset", ctypes.c_size_t), ("len", ctypes.c_size_t)]


VAL_NIL, VAL_BOOL, VAL_INT, VAL_UINT, VAL_FLOAT, VAL_STR, VAL_BIN, VAL_ARRAY, VAL_MAP = range(9)

_P = ctypes.c_void_p
_I32 = ctypes.c_int
_I64 = ctypes.c_int64
_F32 = ctypes.c_float

# name -> (argtypes). Every entry point returns int status.
SIGNATURES = {
    "janus_version": [],
    "janus_stream_create_cu_mask": [_P, _I32, _P],
    "janus_stream_destroy": [_P],
    "janus_duck_pcm16": [_P, _I64, _F32, _P],
    "janus_vad_energy": [_P, _I64, _I32, _I32, _F32, _F32, _P, _P],
    "janus_vad_create": [_P],
    "janus_vad_destroy": [_P],
    "janus_vad_set_tensor": [_P, ctypes.c_char_p, _P, _I64],
    "janus_vad_run": [_P, _P, _I32, _I32, _I32, _I32, _P, _P, _P, _P],
    "janus_prosody_analyze": [_P, _P, _P, _I32, _I64, _I32, _I32, _F32, _F32, _P, _P, _P, _P,
                              _P, _P, _P],
    "janus_prosody_analyze_ex": [_P, _P, _P, _I32, _I64, _I32, _I32, _F32, _F32, _P, _P, _P, _P,
                                 _P, _P, _I32, _P],
    "janus_np_voiced_mean_f32": [_P, _P, _I32, _P, _P, _P],
    "janus_sample_gumbel_f32": [_P, _I32, _I32, _I32, _P, _P],
    "janus_pack_packet": [ctypes.POINTER(janus_packet), _P, ctypes.c_size_t,
                          ctypes.POINTER(ctypes.c_size_t)],
    "janus_unpack": [_P, ctypes.c_size_t, ctypes.POINTER(janus_mp_node), ctypes.c_size_t,
                     ctypes.POINTER(ctypes.c_size_t)],
    "janus_whisper_create": [_P, _P],
    "janus_whisper_destroy": [_P],
    "janus_whisper_set_tensor": [_P, ctypes.c_char_p, _P, _I64],
    "janus_whisper_logmel": [_P, _P, _P, _I32, _I32, _P, _P, _P],
    "janus_whisper_logmel_frames": [_P, _P, _P, _I32, _I32, _I32, _P, _P],
    "janus_whisper_encode": [_P, _P, _I32, _P, _P],
    "janus_whisper_decode_greedy": [_P, _P, _I32, _P, _P, _P, _P, _P],
    "janus_whisper_decode_greedy_ex": [_P, _P, _I32, _P, _P, _P, _P, _P, _P, _P],
    "janus_whisper_decode_sample_ex": [_P, _P, _I32, _P, _P, ctypes.c_float, _P, _P, _P, _P, _P, _P],
    "janus_whisper_decode_sample_rows_ex": [_P, _P, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "janus_whisper_decode_check": [_P, _I32],
    "janus_whisper_decode_info": [_P, _P, _P],
    "janus_whisper_decode_stand": [_P, _P, _I32],
    "janus_whisper_decode_stand_slot": [_P, _I32, _P, _I32],
    "janus_vocoder_create": [_P, _P],
    "janus_vocoder_destroy": [_P],
    "janus_vocoder_set_tensor": [_P, ctypes.c_char_p, _P, _I64],
    "janus_vocoder_frontend": [_P, _P, _P, _P, _I32, _I32, _P, _P],
    "janus_vocoder_frontend_ex": [_P, _P, _P, _P, _P, _I32, _I32, _P, _P],
    "janus_vocoder_speaker": [_P, _P, _P, _I32, _P, _P],
    "janus_vocoder_forward": [_P, _P, _I32, _I32, _P, _P, _P],
    "janus_vocoder_forward_ex": [_P, _P, _I32, _I32, _P, _P, _P, _P],
    "janus_vocoder_set_timing": [_P, _I32],
    "janus_vocoder_conv_stats": [_P, _P, _P, _P, _I32],
    "janus_vocoder_family_stats": [_P, _I32, _P, _P, _P, _P, _P, _P, _I32],
    # include/janus_kernels.h
    "janus_gemm_f16": [_I32, _P, _I64, _P, _I64, _P, _P, _I64, _P, _I64, _I32, _I32, _I32, _P],
    "janus_gemm_nt128_f16": [_I32, _P, _I64, _P, _I64, _P, _P, _I64, _P, _I64, _I32, _I32, _I32, _P],
    "janus_gemm_lt_f16": [_I32, _P, _I64, _P, _I64, _P, _P, _I64, _P, _I64, _I32, _I32, _I32, _P],
    "janus_layernorm_f16": [_P, _P, _P, _P, _I32, _I32, _F32, _P],
    "janus_wave_xor_f32": [_P, _P, _I32, _P],
    "janus_resid_ln_f16": [_P, _I64, _P, _I64, _P, _P, _P, _P, _F32, _P, _I32, _I32, _I32, _P],
    "janus_gemm_ln_f16": [_I32, _P, _I64, _P, _P, _F32, _P, _I64, _P, _P, _I64, _I32, _I32, _I32, _P],
    "janus_attention_f16": [_P, _P, _I32, _I32, _I32, _F32, _P],
    "janus_conv1d_packed_size": [_I32, _I32, _I32, _I32, _I32],
    "janus_conv1d_pack": [_P, _P, _I32, _I32, _I32, _I32, _I32, _P],
    "janus_conv1d_f16": [_P, _I32, _I32, _I32, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _I32,
                         _I32, _I32, _I32, _P, _I64, _F32, _I32, _P],
    "janus_resunit_packed_size": [_I32, _I32],
    "janus_resunit_pack": [_P, _P, _I32, _I32, _P],
    "janus_resunit_f16": [_P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _F32, _I32, _P],
    "janus_cross_attention_f16": [_P, _P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P],
    "janus_decode_attention_f16": [_P, _I64, _P, _P, _I64, _I64, _I32, _P, _I64, _I32, _I32, _F32,
                                   _P, _P, _P],
}
RESTYPES = {"janus_conv1d_packed_size": ctypes.c_int64}

_lib = None


def lib() -> ctypes.CDLL:
    """The loaded library (raises ImportError if it was never built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                "g.build()'` (hipcc --offload-arch=gfx950). janus_amd has no CPU fallback.")
        l = ctypes.CDLL(LIB_PATH)
        l.janus_last_error.restype = ctypes.c_char_p
        l.janus_last_error.argtypes = []
        for name, argtypes in SIGNATURES.items():
            # an A/B build from older sources (JANUS_LIB) may lack the newest test entries
            if os.environ.get("JANUS_LIB") and not hasattr(l, name):
                continue
            fn = getattr(l, name)
            fn.argtypes = argtypes
            fn.restype = RESTYPES.get(name, ctypes.c_int)
        _lib = l
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        raise JanusNativeError(lib().janus_last_error().decode("utf-8", "replace"))


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args))


def require_gpu() -> torch.device:
    """The product path runs on the GPU only; fail loudly otherwise."""
    if not torch.cuda.is_available():
        raise RuntimeError("janus_amd needs an AMD Instinct GPU (gfx950); none is visible")
    lib()
    return torch.device("cuda", torch.cuda.current_device())


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class MaskedStream:
    """A HIP stream restricted to a CU subset (janus_stream_create_cu_mask), usable as a
    torch stream (``torch.cuda.ExternalStream``). ``words``: 32-bit CU mask words."""

    def __init__(self, words, device=None):
        arr = (ctypes.c_uint32 * len(words))(*[int(w) & 0xFFFFFFFF for w in words])
        h = ctypes.c_void_p()
        call("janus_stream_create_cu_mask", ctypes.addressof(arr), len(words), ctypes.addressof(h))
        self._h = h
        self.n_cus = sum(bin(int(w) & 0xFFFFFFFF).count("1") for w in words)
        self.stream = torch.cuda.ExternalStream(h.value, device=device)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().janus_stream_destroy(h)
            except Exception:
                pass


def group_cu_masks(n_cus: int, per_xcd, n_xcd: int = 8):
    """Disjoint CU masks for consecutive groups of per_xcd[g] CUs on every XCD (the same
    interleaved numbering as split_cu_masks: CU i on XCD i % 8, slot i // 8)."""
    slots = n_cus // n_xcd
    assert all(k > 0 for k in per_xcd) and sum(per_xcd) <= slots, (per_xcd, slots)
    words = (n_cus + 31) // 32
    masks = [[0] * words for _ in per_xcd]
    edges = np.cumsum([0] + list(per_xcd))
    for i in range(n_cus):
        g = int(np.searchsorted(edges, i // n_xcd, side="right")) - 1
        if g < len(per_xcd):
            masks[g][i // 32] |= 1 << (i % 32)
    return masks


def split_cu_masks(n_cus: int, dec_per_xcd: int, n_xcd: int = 8):
    """Two disjoint CU masks, balanced per XCD. Workgroups of a launch are dealt round-robin
    to the 8 XCDs whatever the mask, so a launch runs at the pace of the XCD with the
    fewest enabled CUs: each mask must hold the same number of CUs on every XCD. gfx950
    numbers CUs interleaved across XCDs (CU i sits on XCD i % 8; measured: masks that are
    unbalanced under this mapping ran at the speed of their smallest per-XCD share), so
    the first mask takes CU i when (i // 8) < dec_per_xcd, the second the rest."""
    per_xcd = n_cus // n_xcd
    assert 0 < dec_per_xcd < per_xcd, "each side needs at least one CU per XCD"
    words = (n_cus + 31) // 32
    a, b = [0] * words, [0] * words
    for i in range(n_cus):
        if (i // n_xcd) < dec_per_xcd:
            a[i // 32] |= 1 << (i % 32)
        else:
            b[i // 32] |= 1 << (i % 32)
    return a, b
