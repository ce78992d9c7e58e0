"""Wire framing (link_simulator.py:88-116, engine.py:31-52 / :201-218), pinned by the
reference's test_transport_layer.py:233-283 (TCP: 4-byte big-endian length + payload;
UDP: raw bytes)."""
import random
import socket
import struct

from janus_amd.common.wire import FrameReader, frame, frame_batch, recv_exact, recv_packet, transmit_delay


def test_tcp_framing_hello():
    sent = frame(b"hello", use_tcp=True)
    assert len(sent) == 5 + 4
    assert struct.unpack(">I", sent[:4])[0] == 5 and sent[4:] == b"hello"
    assert sent == b"\x00\x00\x00\x05hello"


def test_udp_no_framing():
    assert frame(b"hello world", use_tcp=False) == b"hello world"


def test_transmit_delay_arithmetic():
    # link_simulator.py:100-102: (len + 4) bytes at 300 bps over TCP
    assert abs(transmit_delay(b"x" * 71, True) - 75 / 37.5) < 1e-12
    assert abs(transmit_delay(b"x" * 75, False) - 2.0) < 1e-12


def test_frame_reader_any_slicing():
    rng = random.Random(7)
    payloads = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 300))) for _ in range(40)]
    stream = frame_batch(payloads)
    for trial in range(5):
        r = FrameReader()
        got, i = [], 0
        while i < len(stream):
            j = min(len(stream), i + rng.randrange(1, 97))
            got.extend(r.feed(stream[i:j]))
            i = j
        assert got == payloads and r.pending == 0


def test_recv_exact_and_close():
    a, b = socket.socketpair()
    try:
        a.sendall(frame(b"abc") + frame(b"") + frame(b"xyz" * 1000))
        assert recv_packet(b) == b"abc"
        assert recv_packet(b) == b""
        assert recv_packet(b) == b"xyz" * 1000
        a.sendall(b"\x00\x00\x00\x09par")  # truncated frame, then close
        a.close()
        assert recv_packet(b) is None
        assert recv_exact(b, 1) is None
    finally:
        b.close()
