"""Wire framing of Janus packets.

Sender side, LinkSimulator.transmit (backend/services/link_simulator.py:88-116): over TCP
every MessagePack packet is prefixed with its length as a 4-byte big-endian unsigned int;
over UDP the datagram is the raw packet. Receiver side, receiver_loop
(backend/services/engine.py:31-52 recv_exact, :201-218): read 4 bytes, unpack '>I', read
exactly that many bytes; a closed connection mid-frame ends the stream.

The 300 bps throttle and the progress bar of the simulator are a network demo, not part
of the path (OUT OF SCOPE); ``transmit_delay`` keeps its arithmetic for callers
that want it.
"""
import struct

LENGTH_PREFIX = struct.Struct(">I")
BAUD_RATE = 300                      # link_simulator.py:19
BYTES_PER_SECOND = BAUD_RATE / 8.0   # link_simulator.py:20


def frame(payload: bytes, use_tcp: bool = True) -> bytes:
    """The bytes LinkSimulator.transmit puts on the socket for ``payload``."""
    if not use_tcp:
        return bytes(payload)
    if len(payload) > 0xFFFFFFFF:
        raise ValueError("payload larger than a 4-byte length prefix can describe")
    return LENGTH_PREFIX.pack(len(payload)) + bytes(payload)


def frame_batch(payloads, use_tcp: bool = True) -> bytes:
    """A TCP byte stream carrying ``payloads`` back to back (None entries skipped)."""
    return b"".join(frame(p, use_tcp) for p in payloads if p is not None)


def transmit_delay(payload: bytes, use_tcp: bool = True) -> float:
    """Seconds the simulator sleeps for one transmit (link_simulator.py:100-102)."""
    return len(frame(payload, use_tcp)) / BYTES_PER_SECOND


def recv_exact(sock, n: int):
    """engine.py:31-52: exactly n bytes from a stream socket, or None if it closes first."""
    buf = bytearray()
    while len(buf) < n:
        part = sock.recv(n - len(buf))
        if not part:
            return None
        buf.extend(part)
    return bytes(buf)


def recv_packet(sock):
    """One framed packet from a TCP socket (engine.py:201-218), or None on close."""
    head = recv_exact(sock, 4)
    if head is None:
        return None
    (n,) = LENGTH_PREFIX.unpack(head)
    return recv_exact(sock, n)


class FrameReader:
    """Incremental decoder of a length-prefixed TCP byte stream: feed() arbitrary slices
    of the stream, get back every packet completed so far (the receiver's recv_exact loop
    without a socket, e.g. for a batched receiver draining many connections)."""

    def __init__(self):
        self._buf = bytearray()

    def feed(self, data: bytes):
        self._buf.extend(data)
        out = []
        while len(self._buf) >= 4:
            (n,) = LENGTH_PREFIX.unpack_from(self._buf, 0)
            if len(self._buf) < 4 + n:
                break
            out.append(bytes(self._buf[4:4 + n]))
            del self._buf[:4 + n]
        return out

    @property
    def pending(self) -> int:
        """Bytes of an incomplete frame still buffered."""
        return len(self._buf)
