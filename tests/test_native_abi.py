"""The C-ABI library loads and exports every symbol include/janus.h declares (CPU)."""
import ctypes
import os
import re

from janus_amd import _native

HEADER_DIR = os.path.join(os.path.dirname(__file__), "..", "include")


def declared_symbols():
    names = set()
    for fn in os.listdir(HEADER_DIR):
        if fn.endswith(".h"):
            src = open(os.path.join(HEADER_DIR, fn)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names |= set(re.findall(r"\b(janus_[a-z0-9_]+)\s*\(", src))
    return names


def test_header_symbols_exported(native_lib):
    names = declared_symbols()
    assert "janus_prosody_analyze" in names and "janus_pack_packet" in names
    for name in sorted(names):
        assert hasattr(native_lib, name), f"{name} declared in include/ but not exported"


def test_python_signatures_cover_header(native_lib):
    names = declared_symbols() - {"janus_last_error"}
    missing = names - set(_native.SIGNATURES)
    assert not missing, f"no ctypes signature for {sorted(missing)}"


def test_version_and_error_slot(native_lib):
    assert native_lib.janus_version() >= 100
    assert isinstance(native_lib.janus_last_error(), bytes)


def test_gfx950_code_object():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_split_cu_masks_balanced_per_xcd():
    """Both masks of the overlapped step hold the same CU count on every XCD (CU i on XCD
    i % 8) and, at multiples of 4, on every shader engine; they are disjoint and cover
    all CUs."""
    for dec in (4, 8, 16, 20, 28):
        a, b = _native.split_cu_masks(256, dec)
        bits_a = [i for i in range(256) if a[i // 32] >> (i % 32) & 1]
        bits_b = [i for i in range(256) if b[i // 32] >> (i % 32) & 1]
        assert len(bits_a) == 8 * dec and len(bits_a) + len(bits_b) == 256
        assert not set(bits_a) & set(bits_b)
        for x in range(8):
            assert sum(1 for i in bits_a if i % 8 == x) == dec


def test_group_cu_masks_three_lanes():
    """The three-lane step's masks (decoder, encoder, vocoder): disjoint, balanced per XCD,
    cover exactly the requested counts; two groups reproduce split_cu_masks."""
    for per in ([12, 4, 16], [14, 2, 16], [16, 4, 12], [8, 8, 8]):
        masks = _native.group_cu_masks(256, per)
        seen = set()
        for m, k in zip(masks, per):
            bits = [i for i in range(256) if m[i // 32] >> (i % 32) & 1]
            assert len(bits) == 8 * k and not seen & set(bits)
            seen |= set(bits)
            for x in range(8):
                assert sum(1 for i in bits if i % 8 == x) == k
    for dec in (4, 16, 28):
        assert _native.group_cu_masks(256, [dec, 32 - dec]) == list(_native.split_cu_masks(256, dec))
