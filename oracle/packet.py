"""ORACLE — test infrastructure only (see oracle/__init__.py).

Byte-level restatement of the Janus packet wire format: ``JanusPacket.to_dict``
(backend/common/protocol.py:57-76) encoded the way ``msgpack.packb(...,
use_bin_type=True)`` (:107) encodes it, written from the MessagePack spec
(fixmap/fixstr/str8/16/32, fix/u/int 8-64, float64). Independent of the msgpack
package so the two can check each other. Pinned by the spec-level vectors
recorded in SURVEY.md §8(a9)/(c) (tests/golden/packets.json) and by the
reference's tests test_transport_layer.py:29-147.
"""
import struct


def _str(s: str) -> bytes:
    b = s.encode('utf-8')
    n = len(b)
    if n < 32:
        return bytes([0xa0 | n]) + b
    if n < 256:
        return b'\xd9' + bytes([n]) + b
    if n < 65536:
        return b'\xda' + struct.pack('>H', n) + b
    return b'\xdb' + struct.pack('>I', n) + b


def _int(v: int) -> bytes:
    if v >= 0:
        if v < 128:
            return bytes([v])
        if v <= 0xff:
            return b'\xcc' + struct.pack('>B', v)
        if v <= 0xffff:
            return b'\xcd' + struct.pack('>H', v)
        if v <= 0xffffffff:
            return b'\xce' + struct.pack('>I', v)
        return b'\xcf' + struct.pack('>Q', v)
    if v >= -32:
        return struct.pack('>b', v)
    if v >= -128:
        return b'\xd0' + struct.pack('>b', v)
    if v >= -32768:
        return b'\xd1' + struct.pack('>h', v)
    if v >= -2 ** 31:
        return b'\xd2' + struct.pack('>i', v)
    return b'\xd3' + struct.pack('>q', v)


def _map_header(n: int) -> bytes:
    if n < 16:
        return bytes([0x80 | n])
    if n < 65536:
        return b'\xde' + struct.pack('>H', n)
    return b'\xdf' + struct.pack('>I', n)


def _value(v) -> bytes:
    if v is None:
        return b'\xc0'
    if v is True:
        return b'\xc3'
    if v is False:
        return b'\xc2'
    if isinstance(v, int):
        return _int(int(v))
    if isinstance(v, float):
        return b'\xcb' + struct.pack('>d', v)
    if isinstance(v, str):
        return _str(str(v))
    if isinstance(v, dict):
        return _map_header(len(v)) + b''.join(_str(k) + _value(x) for k, x in v.items())
    raise TypeError(f"oracle packer: unsupported type {type(v)}")


def to_dict(text, mode, prosody, override_emotion, timestamp) -> dict:
    """protocol.py:57-76 (override default "Auto" applied by the caller, :53)."""
    d = {'t': text, 'm': int(mode), 'p': prosody, 'ts': timestamp}
    if override_emotion != "Auto":
        d['o'] = override_emotion
    return d


def serialize(text, mode, prosody, override_emotion="Auto", timestamp=0.0) -> bytes:
    return _value(to_dict(text, mode, prosody, override_emotion, timestamp))
