"""Generates tests/golden/packets.json (run from the repo root).

Expected bytes come from the oracle's spec restatement (oracle/packet.py) and are
cross-checked against the msgpack package (third-party, 1.2.1 here; the library the
reference calls at backend/common/protocol.py:107). The first three cases are the
hand-decoded spec-level vectors recorded in SURVEY.md §8(c); the rest cover every
length/int form the codec can emit (fixstr/str8/str16, fixint/uint8/16/32/64,
negative ints, float64 vs int timestamps, UTF-8 text, empty prosody, 'o' present).
"""
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import msgpack  # noqa: E402

from oracle import packet as op  # noqa: E402

CASES = [
    # 58 B
    dict(text="Hello world", mode=0, prosody={"energy": "Normal", "pitch": "High"},
         override="Auto", ts=1234567890.0,
         expect="84a174ab48656c6c6f20776f726c64a16d00a17082a6656e65726779a64e6f726d616c"
                "a57069746368a448696768a27473cb41d26580b4800000"),
    # engine path: 'o': 'auto' (engine.py:542-547 with control_state.emotion_override)
    dict(text="Hello world", mode=0, prosody={"energy": "Normal", "pitch": "High"},
         override="auto", ts=1234567890.0,
         expect="85a174ab48656c6c6f20776f726c64a16d00a17082a6656e65726779a64e6f726d616c"
                "a57069746368a448696768a27473cb41d26580b4800000a16fa46175746f"),
    dict(text="x" * 40, mode=1, prosody={}, override="Auto", ts=1.5,
         expect="84a174d928" + "78" * 40 + "a16d01a17080a27473cb3ff8000000000000"),
    dict(text="", mode=2, prosody={}, override="Auto", ts=0.0),
    dict(text="reconstructed text", mode=2, prosody={"energy": "Quiet", "pitch": "Normal"},
         override="Joyful", ts=9999999999.0),
    dict(text="test", mode=1, prosody={"energy": "Loud", "pitch": "Deep"}, override="Panicked",
         ts=1700000000.123456),
    dict(text="y" * 31, mode=0, prosody={"energy": "Normal", "pitch": "Normal"}, override="Auto",
         ts=2.0),
    dict(text="z" * 255, mode=0, prosody={"pitch": "High", "energy": "Loud"}, override="Auto",
         ts=3.0),
    dict(text="w" * 256, mode=0, prosody={"energy": "Loud"}, override="excited", ts=4.0),
    dict(text="v" * 70000, mode=0, prosody={}, override="Auto", ts=5.0),
    dict(text="héllo wörld ☺ \U0001f600", mode=0,
         prosody={"energy": "Normal", "pitch": "Deep"}, override="Auto", ts=-1.25),
    dict(text="int ts", mode=0, prosody={}, override="Auto", ts=1700000000),
    dict(text="neg ts", mode=0, prosody={}, override="Auto", ts=-5),
    dict(text="int forms", mode=0,
         prosody={"a": 127, "b": 128, "c": 255, "d": 256, "e": 65535, "f": 65536,
                  "g": 4294967295, "h": 4294967296, "i": -1, "j": -32, "k": -33, "l": -128,
                  "m": -129, "n": -32768, "o": -32769, "p": -2147483648, "q": -2147483649,
                  "r": 2 ** 63 - 1},
         override="Auto", ts=6.0),
    dict(text="scalars", mode=0, prosody={"avg_pitch_hz": 151.25, "flag": True, "none": None,
                                          "off": False}, override="Auto", ts=7.0),
]


def main():
    out = []
    for c in CASES:
        ours = op.serialize(c["text"], c["mode"], c["prosody"], c["override"], c["ts"])
        ref = msgpack.packb(op.to_dict(c["text"], c["mode"], c["prosody"], c["override"], c["ts"]),
                            use_bin_type=True)
        assert ours == ref, (c["text"][:20], ours.hex(), ref.hex())
        if "expect" in c:
            assert ours.hex() == c["expect"], (ours.hex(), c["expect"])
        out.append(dict(text=c["text"], mode=c["mode"], prosody=c["prosody"],
                        override=c["override"], ts=c["ts"], hex=ours.hex()))
    path = os.path.join(os.path.dirname(__file__), "packets.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, ensure_ascii=True)
    print(f"wrote {len(out)} packet vectors to {path}")


if __name__ == "__main__":
    main()
