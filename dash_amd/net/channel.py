"""Length-prefixed message framing over TCP.

Frame: 4-byte ASCII tag, u32 flags, u64 payload length, payload. Payloads are
sent with sendall from memoryviews (no extra copy for numpy buffers) and
received into one preallocated bytearray. Every operation has a timeout so a
dead peer surfaces as an exception instead of a hang.
"""
from __future__ import annotations

import socket
import struct
from typing import Optional, Tuple

_HDR = struct.Struct("<4sIQ")
MAX_FRAME = 1 << 40


class ChannelClosed(ConnectionError):
    pass


class Channel:
    def __init__(self, sock: socket.socket, timeout: Optional[float] = 600.0):
        self.sock = sock
        self.sock.settimeout(timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.bytes_sent = 0
        self.bytes_recv = 0

    def send(self, tag: bytes, payload=b"", flags: int = 0) -> None:
        assert len(tag) == 4
        mv = memoryview(payload).cast("B") if not isinstance(payload, (bytes, bytearray)) else memoryview(payload)
        self.sock.sendall(_HDR.pack(tag, flags, mv.nbytes))
        if mv.nbytes:
            self.sock.sendall(mv)
        self.bytes_sent += _HDR.size + mv.nbytes

    def _recv_into(self, buf: memoryview) -> None:
        got = 0
        while got < len(buf):
            n = self.sock.recv_into(buf[got:], len(buf) - got)
            if n == 0:
                raise ChannelClosed("peer closed the connection")
            got += n

    def recv(self, expect: Optional[bytes] = None) -> Tuple[bytes, int, bytearray]:
        hdr = bytearray(_HDR.size)
        self._recv_into(memoryview(hdr))
        tag, flags, n = _HDR.unpack(hdr)
        if n > MAX_FRAME:
            raise ValueError(f"frame too large: {n}")
        buf = bytearray(n)
        if n:
            self._recv_into(memoryview(buf))
        self.bytes_recv += _HDR.size + n
        if tag == b"ERR!":
            raise RuntimeError("peer error: " + buf.decode(errors="replace"))
        if expect is not None and tag != expect:
            raise ValueError(f"protocol: expected {expect!r}, got {tag!r}")
        return tag, flags, buf

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def listen(host: str = "127.0.0.1", port: int = 0) -> socket.socket:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.bind((host, port))
    s.listen(1)
    return s


def connect(host: str, port: int, timeout: float = 600.0, retries: int = 50) -> Channel:
    import time

    last = None
    for _ in range(retries):
        try:
            return Channel(socket.create_connection((host, port), timeout=timeout), timeout)
        except OSError as e:  # server not up yet
            last = e
            time.sleep(0.1)
    raise ConnectionError(f"cannot connect to {host}:{port}: {last}")
