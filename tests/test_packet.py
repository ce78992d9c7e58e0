"""Packet codec parity: native janus_pack_packet/janus_unpack vs golden vectors,
the oracle restatement and msgpack (CPU; host code, no GPU needed).
Mirrors backend/tests/test_transport_layer.py:26-147."""
import json
import os
import time

import msgpack
import pytest

from janus_amd.common.protocol import JanusMode, JanusPacket, unpack
from oracle import packet as op

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "packets.json")))


@pytest.mark.parametrize("case", GOLDEN, ids=lambda c: c["text"][:12] or "empty")
def test_golden_bytes(native_lib, case):
    pkt = JanusPacket(case["text"], JanusMode(case["mode"]), case["prosody"], case["override"],
                      case["ts"])
    data = pkt.serialize()
    assert data.hex() == case["hex"]
    assert data == op.serialize(case["text"], case["mode"], case["prosody"], case["override"],
                                case["ts"])
    back = JanusPacket.deserialize(data)
    assert back.text == case["text"] and back.mode == case["mode"]
    assert back.prosody == case["prosody"]
    assert back.override_emotion == case["override"]
    assert back.timestamp == case["ts"]
    assert unpack(data) == msgpack.unpackb(data, raw=False)


def test_serialization_cycle(native_lib):
    p = JanusPacket("Hello world", JanusMode.SEMANTIC_VOICE, {'energy': 'Normal', 'pitch': 'High'},
                    override_emotion="Relaxed", timestamp=1234567890.0)
    d = JanusPacket.deserialize(p.serialize())
    assert (d.text, d.mode, d.prosody, d.override_emotion, d.timestamp) == \
        ("Hello world", JanusMode.SEMANTIC_VOICE, {'energy': 'Normal', 'pitch': 'High'},
         "Relaxed", 1234567890.0)


def test_compact_keys_and_override_rule(native_lib):
    p = JanusPacket("test", JanusMode.TEXT_ONLY, {'energy': 'Loud', 'pitch': 'Deep'},
                    override_emotion="Panicked")
    d = p.to_dict()
    assert set(d) == {'t', 'm', 'p', 'ts', 'o'} and d['m'] == 1
    assert 'o' not in JanusPacket("t", JanusMode.SEMANTIC_VOICE, {}, "Auto").to_dict()
    assert 'o' not in unpack(JanusPacket("t", JanusMode.SEMANTIC_VOICE, {}, "Auto").serialize())


@pytest.mark.parametrize("garbage", [b'\x00\x01\x02\x03\xff\xfe\xfd', b'', b'\xc1', b'\x85\xa1',
                                     b'\xd9\x05ab', b'\x81\x01\x02'])
def test_deserialize_garbage_raises(native_lib, garbage):
    with pytest.raises(Exception):
        JanusPacket.deserialize(garbage)
    with pytest.raises(Exception):
        msgpack.unpackb(garbage, raw=False)


def test_from_dict_and_timestamp_default(native_lib):
    p = JanusPacket.from_dict({'t': 'reconstructed text', 'm': 2,
                               'p': {'energy': 'Quiet', 'pitch': 'Normal'}, 'o': 'Joyful',
                               'ts': 9999999999.0})
    assert p.mode == JanusMode.MORSE_CODE and p.timestamp == 9999999999.0
    assert abs(JanusPacket("t", JanusMode.SEMANTIC_VOICE, {}).timestamp - time.time()) < 1.0


def test_str_enum_override_packs_as_str(native_lib):
    import enum

    class Emotion(str, enum.Enum):
        AUTO = "auto"

    p = JanusPacket("Hello world", JanusMode.SEMANTIC_VOICE, {'energy': 'Normal', 'pitch': 'High'},
                    Emotion.AUTO, 1234567890.0)
    assert p.serialize() == msgpack.packb(p.to_dict(), use_bin_type=True)


def test_unsupported_type_raises(native_lib):
    with pytest.raises(TypeError):
        JanusPacket("x", 0, {'energy': object()}, timestamp=1.0).serialize()


def test_str_subclass_values_pack_by_value(native_lib):
    """str-enum prosody keys/values, text and override (a caller's `class Tag(str, Enum)`)
    pack as their string value, byte for byte what msgpack 1.2.1 emits for the reference's
    to_dict (protocol.py:107); str(member) would be "Tag.NORMAL" on Python 3.10."""
    import enum

    class Tag(str, enum.Enum):
        ENERGY = "energy"
        PITCH = "pitch"
        NORMAL = "Normal"
        HIGH = "High"

    class Text(str):
        def __str__(self):
            return "not this"

    for override in ("Auto", Text("(joyful)")):
        pkt = JanusPacket(Text("Hello world"), JanusMode.SEMANTIC_VOICE,
                          {Tag.ENERGY: Tag.NORMAL, Tag.PITCH: Tag.HIGH}, override, 1234567890.0)
        ref = {'t': Text("Hello world"), 'm': 0, 'p': {Tag.ENERGY: Tag.NORMAL, Tag.PITCH: Tag.HIGH},
               'ts': 1234567890.0}
        if override != "Auto":
            ref['o'] = override
        assert pkt.serialize() == msgpack.packb(ref, use_bin_type=True)
    plain = JanusPacket("Hello world", JanusMode.SEMANTIC_VOICE, {'energy': 'Normal', 'pitch': 'High'},
                        None, 1234567890.0)
    tagged = JanusPacket("Hello world", JanusMode.SEMANTIC_VOICE,
                         {Tag.ENERGY: Tag.NORMAL, Tag.PITCH: Tag.HIGH}, None, 1234567890.0)
    assert tagged.serialize() == plain.serialize()
