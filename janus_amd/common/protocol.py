"""Janus packet schema and wire codec — drop-in for backend/common/protocol.py.

Same names, argument meaning and error behaviour as the reference
(``JanusMode`` :15-21, ``JanusPacket`` :24-121); the MessagePack encode/decode that
the reference delegates to the msgpack C extension (:107, :120) runs in
libjanus_hip.so (``janus_pack_packet`` / ``janus_unpack``, include/janus.h).
"""
import ctypes
import enum
import threading
import time
from typing import Optional

from .. import _native as nat


class JanusMode(enum.IntEnum):
    """Transmission modes (protocol.py:15-21)."""
    SEMANTIC_VOICE = 0
    TEXT_ONLY = 1
    MORSE_CODE = 2


def _to_value(v, keep) -> nat.janus_value:
    """Python scalar -> janus_value with msgpack-python's type rules (bool before int,
    Python float incl. numpy.float64 -> float64, other types rejected)."""
    out = nat.janus_value()
    if v is None:
        out.type = nat.VAL_NIL
    elif v is True or v is False:
        out.type, out.i = nat.VAL_BOOL, int(v)
    elif isinstance(v, int):
        iv = int(v)
        if iv > 2 ** 63 - 1:
            if iv >= 2 ** 64:
                raise OverflowError("Integer value out of range")
            out.type, out.i = nat.VAL_UINT, iv - 2 ** 64
        else:
            if iv < -2 ** 63:
                raise OverflowError("Integer value out of range")
            out.type, out.i = nat.VAL_INT, iv
    elif isinstance(v, float):
        out.type, out.f = nat.VAL_FLOAT, float(v)
    elif isinstance(v, str):
        # by value, as msgpack packs any str subclass (str(v) of a str-enum member is
        # "Cls.MEMBER" on Python 3.10; protocol.py:107 packs the member's value)
        b = str.encode(v, "utf-8")
        keep.append(b)
        out.type, out.s, out.len = nat.VAL_STR, b, len(b)
    else:
        raise TypeError(f"can not serialize {type(v).__name__!r} object in a Janus packet")
    return out


def pack_dict_fields(text, mode, prosody, override, timestamp) -> bytes:
    """Encode the packet map (t, m, p, ts[, o]) through janus_pack_packet."""
    keep = []
    if not isinstance(text, str):
        raise TypeError("packet text must be str")
    tb = str.encode(text, "utf-8")
    items = list((prosody or {}).items()) if prosody is not None else []
    if prosody is not None and not isinstance(prosody, dict):
        raise TypeError("prosody must be a dict")
    n = len(items)
    keys = (nat.janus_value * max(n, 1))()
    vals = (nat.janus_value * max(n, 1))()
    for k, (key, val) in enumerate(items):
        if not isinstance(key, str):
            raise TypeError("prosody keys must be str")
        keys[k] = _to_value(key, keep)
        vals[k] = _to_value(val, keep)
    pkt = nat.janus_packet()
    pkt.text, pkt.text_len = tb, len(tb)
    pkt.mode = int(mode)
    pkt.n_prosody = n
    pkt.prosody_keys = ctypes.cast(keys, ctypes.POINTER(nat.janus_value))
    pkt.prosody_vals = ctypes.cast(vals, ctypes.POINTER(nat.janus_value))
    if override is not None:
        if not isinstance(override, str):
            raise TypeError("override_emotion must be str")
        ob = str.encode(override, "utf-8")
        keep.append(ob)
        pkt.override_emotion, pkt.override_len = ob, len(ob)
    else:
        pkt.override_emotion, pkt.override_len = None, 0
    if isinstance(timestamp, bool) or not isinstance(timestamp, (int, float)):
        raise TypeError("timestamp must be float or int")
    pkt.timestamp = _to_value(timestamp, keep)
    cap = 64 + len(tb) + 2 * sum(len(b) for b in keep) + 32 * n
    buf = (ctypes.c_uint8 * cap)()
    out_len = ctypes.c_size_t(0)
    nat.call("janus_pack_packet", ctypes.byref(pkt), buf, cap, ctypes.byref(out_len))
    return bytes(buf[:out_len.value])


_tls = threading.local()


def _node_buffer(cap: int):
    """Per-thread reusable node array (allocating and zeroing a fresh ctypes array of
    len(payload) nodes per call cost ~1 ms for a 2 KB transcript)."""
    buf = getattr(_tls, "nodes", None)
    if buf is None or len(buf) < cap:
        buf = (nat.janus_mp_node * max(cap, 1024))()
        _tls.nodes = buf
    return buf


def unpack(payload: bytes):
    """msgpack.unpackb(payload, raw=False) semantics via janus_unpack."""
    if not isinstance(payload, (bytes, bytearray, memoryview)):
        raise TypeError("a bytes-like object is required")
    payload = bytes(payload)
    cap = len(payload) + 1  # every MessagePack object takes >= 1 byte
    nodes = _node_buffer(cap)
    n = ctypes.c_size_t(0)
    src = ctypes.create_string_buffer(payload, len(payload)) if payload else None
    nat.call("janus_unpack", src, len(payload), nodes, cap, ctypes.byref(n))

    pos = 0

    def build():
        nonlocal pos
        nd = nodes[pos]
        pos += 1
        t = nd.type
        if t == nat.VAL_NIL:
            return None
        if t == nat.VAL_BOOL:
            return bool(nd.i)
        if t == nat.VAL_INT:
            return int(nd.i)
        if t == nat.VAL_UINT:
            return int(nd.i) + 2 ** 64
        if t == nat.VAL_FLOAT:
            return float(nd.f)
        if t == nat.VAL_STR:
            return payload[nd.offset:nd.offset + nd.len].decode("utf-8")
        if t == nat.VAL_BIN:
            return payload[nd.offset:nd.offset + nd.len]
        if t == nat.VAL_ARRAY:
            return [build() for _ in range(nd.len)]
        if t == nat.VAL_MAP:
            d = {}
            for _ in range(nd.len):
                k = build()
                if not isinstance(k, (str, bytes)):
                    raise ValueError(f"{type(k).__name__} is not allowed for map key")
                d[k] = build()
            return d
        raise ValueError(f"unexpected node type {t}")

    return build()


class JanusPacket:
    """The packet (protocol.py:24-121), compact keys t/m/p/o/ts."""

    def __init__(self, text: str, mode: JanusMode, prosody: dict[str, str],
                 override_emotion: Optional[str] = None,
                 timestamp: Optional[float] = None) -> None:
        self.text = text
        self.mode = mode
        self.prosody = prosody
        self.override_emotion = override_emotion if override_emotion is not None else "Auto"
        self.timestamp = timestamp if timestamp is not None else time.time()

    def to_dict(self) -> dict:
        result = {
            't': self.text,
            'm': int(self.mode),
            'p': self.prosody,
            'ts': self.timestamp,
        }
        if self.override_emotion != "Auto":
            result['o'] = self.override_emotion
        return result

    @classmethod
    def from_dict(cls, data: dict) -> "JanusPacket":
        text = data.get('t', '')
        mode = JanusMode(data.get('m', 0))
        prosody = data.get('p', {})
        override_emotion = data.get('o', 'Auto')
        timestamp = data.get('ts', time.time())
        return cls(text, mode, prosody, override_emotion, timestamp)

    def serialize(self) -> bytes:
        override = self.override_emotion if self.override_emotion != "Auto" else None
        return pack_dict_fields(self.text, self.mode, self.prosody, override, self.timestamp)

    @classmethod
    def deserialize(cls, payload_bytes: bytes) -> "JanusPacket":
        return cls.from_dict(unpack(payload_bytes))
