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


def _c_offsets(struct, fields):
    """offsetof() of each field of a header struct, from a C program gcc builds here."""
    import shutil
    import subprocess
    import tempfile
    import pytest
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    body = "".join(f'  printf("%zu\\n", offsetof({struct}, {f}));\n' for f in fields)
    src = ("#include <stddef.h>\n#include <stdio.h>\n#include \"janus.h\"\n"
           f"int main(void) {{\n{body}  printf(\"%zu\\n\", sizeof({struct}));\n  return 0;\n}}\n")
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "o.c"), os.path.join(d, "o")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", HEADER_DIR, c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    return [int(v) for v in out]


def test_decode_structs_match_header():
    """The ctypes mirrors of janus_decode_options / janus_decode_rows lay out exactly as the
    C header (field offsets and size), so every option reaches the library."""
    from janus_amd.whisper import janus_decode_options, janus_decode_rows
    for cls in (janus_decode_options, janus_decode_rows):
        names = [n for n, _ in cls._fields_]
        want = _c_offsets(cls.__name__, names)
        got = [getattr(cls, n).offset for n in names] + [ctypes.sizeof(cls)]
        assert got == want, (cls.__name__, got, want)


def test_decode_path_flags_match_header():
    from janus_amd import whisper as w
    src = open(os.path.join(HEADER_DIR, "janus.h")).read()
    flags = dict(re.findall(r"#define JANUS_DEC_PATH_([A-Z0-9_]+)\s+(0x[0-9a-fA-F]+)u", src))
    assert len(flags) == 14
    for name, v in flags.items():
        assert getattr(w, "DEC_PATH_" + name) == int(v, 16), name
    assert w.dec_path_ln_mask(9) == 0x0800 | (9 << 12)


def test_product_library_reads_no_tuning_environment():
    """Kernel-geometry A/B switches exist only in -DJANUS_AB_KNOBS builds (common.h ab_env):
    the product library carries no JANUS_* environment name."""
    data = open(_native.LIB_PATH, "rb").read()
    assert not re.findall(rb"JANUS_[A-Z0-9_]+\x00", data)
