"""asyncio front-end for the native uTP engine (``tritondl._utp``, C++).

One UDP socket per :class:`UtpSocket` multiplexes every uTP connection (as
libutp / anacrolix do, sharing the BitTorrent listen port number).  Each
connection is exposed as a standard ``(asyncio.StreamReader,
asyncio.StreamWriter)`` pair, so the peer-wire code runs unchanged over TCP
or uTP.  Python never touches individual datagrams: the event loop only
reports the socket readable/writable and the native ``Pump`` drains it with
recvmmsg / sendmmsg; sequencing, SACK, RTO and LEDBAT live in C++.
"""

from __future__ import annotations

import asyncio
import contextlib
import socket
import time
from typing import Callable

try:
    from ... import _utp  # type: ignore[attr-defined]
except ImportError as e:  # pragma: no cover - built by tools/build_native.py
    raise ImportError("tritondl native uTP extension is not built; run `python tools/build_native.py`") from e

TICK = 0.01
HIGH_WATER = 1 << 20


def _now_us() -> int:
    return time.monotonic_ns() // 1000


def _key(addr: tuple[str, int]) -> str:
    return f"{addr[0]}:{addr[1]}"


def _addr(key: str) -> tuple[str, int]:
    h, _, p = key.rpartition(":")
    return h, int(p)


class UtpError(ConnectionError):
    pass


class _UtpTransport(asyncio.Transport):
    def __init__(self, sock: "UtpSocket", cid: int, peer: tuple[str, int]) -> None:
        super().__init__()
        self.sock = sock
        self.cid = cid
        self.peer = peer
        self._closing = False
        self._buf = bytearray()
        self._protocol: asyncio.Protocol | None = None
        self._paused = False

    def get_extra_info(self, name, default=None):
        if name == "peername":
            return self.peer
        if name == "sockname":
            return self.sock.local_addr
        if name == "socket":
            return None
        return default

    def is_closing(self) -> bool:
        return self._closing

    def set_protocol(self, protocol) -> None:
        self._protocol = protocol

    def get_protocol(self):
        return self._protocol

    def write(self, data) -> None:
        if self._closing:
            return
        self._buf += data
        self._push()
        self.sock._flush()

    def _push(self) -> None:
        eng = self.sock.engine
        if self._buf:
            n = eng.write(self.cid, bytes(self._buf[:HIGH_WATER]))
            if n:
                del self._buf[:n]
        pend = len(self._buf) + eng.send_buffered(self.cid)
        if self._protocol is not None:
            if not self._paused and pend > 4 * HIGH_WATER:
                self._paused = True
                self._protocol.pause_writing()
            elif self._paused and pend < HIGH_WATER:
                self._paused = False
                self._protocol.resume_writing()

    def pause_reading(self) -> None:
        """Leave delivered bytes in the engine: its advertised receive window
        closes as they pile up, so the peer stops sending (real backpressure,
        not an unbounded buffer on our side)."""
        self.stream.paused = True

    def resume_reading(self) -> None:
        if self.stream.paused:
            self.stream.paused = False
            self.sock._service(self.cid)       # hand over what waited (and reopen the window)
            self.sock._flush()

    def is_reading(self) -> bool:
        return not self.stream.paused

    def can_write_eof(self) -> bool:
        return False

    def get_write_buffer_size(self) -> int:
        return len(self._buf) + self.sock.engine.send_buffered(self.cid)

    def close(self) -> None:
        if self._closing:
            return
        self._closing = True
        if self._buf:
            self.sock.engine.write(self.cid, bytes(self._buf))
            self._buf.clear()
        self.sock.engine.close(self.cid, _now_us())
        self.sock.engine.forget(self.cid)
        self.sock._flush()

    def abort(self) -> None:
        self._closing = True
        self.sock.engine.abort(self.cid)
        self.sock.engine.forget(self.cid)
        self.sock._flush()


class _Stream:
    def __init__(self, sock: "UtpSocket", cid: int, peer: tuple[str, int]) -> None:
        loop = asyncio.get_running_loop()
        self.reader = asyncio.StreamReader(limit=1 << 22)
        self.protocol = asyncio.StreamReaderProtocol(self.reader)
        self.transport = _UtpTransport(sock, cid, peer)
        self.transport.stream = self
        self.transport.set_protocol(self.protocol)
        self.protocol.connection_made(self.transport)
        self.writer = asyncio.StreamWriter(self.transport, self.protocol, self.reader, loop)
        self.connected = asyncio.Event()
        self.eof = False
        # a native link's receive hook (peer.Wire.take_over): when set, bytes
        # the engine delivers go straight to it instead of the StreamReader
        self.sink: Callable[[bytes], None] | None = None
        self.sink_eof: Callable[[], None] | None = None
        self.paused = False        # the reader is backed up: bytes stay in the engine


class UtpSocket:
    def __init__(self, seed: int = 0) -> None:
        self.engine = _utp.Engine(seed)
        self._sock: socket.socket | None = None
        self._pump = None
        self._writing = False
        self.streams: dict[int, _Stream] = {}
        self.accept_q: asyncio.Queue = asyncio.Queue()
        self.local_addr: tuple[str, int] = ("0.0.0.0", 0)
        self._ticker: asyncio.Task | None = None
        self._loop: asyncio.AbstractEventLoop | None = None
        self.other_datagram = None   # optional handler for non-uTP datagrams (e.g. DHT on a shared port)

    async def start(self, host: str = "0.0.0.0", port: int = 0) -> "UtpSocket":
        self._loop = asyncio.get_running_loop()
        fam = socket.AF_INET6 if ":" in host else socket.AF_INET
        sock = socket.socket(fam, socket.SOCK_DGRAM)
        sock.setblocking(False)
        for opt in (socket.SO_RCVBUF, socket.SO_SNDBUF):
            with contextlib.suppress(OSError):
                sock.setsockopt(socket.SOL_SOCKET, opt, 8 << 20)   # capped by rmem_max/wmem_max
        try:
            sock.bind((host, port))
        except OSError:
            sock.close()
            raise
        self._sock = sock
        self._pump = _utp.Pump(self.engine, sock.fileno())
        self.local_addr = sock.getsockname()[:2]
        self._loop.add_reader(sock.fileno(), self._on_readable)
        self._ticker = asyncio.ensure_future(self._tick_loop())
        return self

    @property
    def port(self) -> int:
        return self.local_addr[1]

    def close(self) -> None:
        for s in list(self.streams.values()):
            if not s.transport.is_closing():
                s.transport.abort()
            if not s.eof:
                s.eof = True
                s.reader.feed_eof()
                if s.sink_eof is not None:
                    s.sink_eof()
        self._flush()
        if self._ticker is not None:
            self._ticker.cancel()
        if self._sock is not None:
            with contextlib.suppress(Exception):
                self._loop.remove_reader(self._sock.fileno())   # type: ignore[union-attr]
                self._loop.remove_writer(self._sock.fileno())   # type: ignore[union-attr]
            self._sock.close()
            self._sock = None

    # ------------------------------------------------------------ io
    def _on_readable(self) -> None:
        if self._sock is None:
            return
        touched, others = self._pump.recv(_now_us())
        for new in self.engine.accepted():
            st = self.stats(new)
            s = _Stream(self, new, _addr(st["addr"]))
            s.connected.set()
            self.streams[new] = s
            self.accept_q.put_nowait(s)
        for cid in touched:
            self._service(cid)
        if others and self.other_datagram is not None:
            for data, addr in others:
                self.other_datagram(data, addr)
        self._flush()

    def datagram_received(self, data: bytes, addr) -> None:
        """Feed one datagram by hand (tests / a foreign socket owner)."""
        cid = self.engine.incoming(data, _key(addr[:2]), _now_us())
        for new in self.engine.accepted():
            s = _Stream(self, new, _addr(self.stats(new).get("addr", _key(addr[:2]))))
            s.connected.set()
            self.streams[new] = s
            self.accept_q.put_nowait(s)
        if cid > 0:
            self._service(cid)
        self._flush()

    def error_received(self, exc: Exception) -> None:  # ICMP errors etc.
        pass

    def _service(self, cid: int) -> None:
        s = self.streams.get(cid)
        if s is None:
            return
        st = self.engine.state(cid)
        if st >= _utp.CONNECTED and not s.connected.is_set() and st != _utp.RESET:
            s.connected.set()
        if s.paused and st != _utp.RESET:
            s.transport._push()           # keep sending; receive resumes on resume_reading()
            return
        data = self.engine.read(cid)
        if data:
            if s.sink is not None:
                s.sink(data)
            else:
                s.reader.feed_data(data)
        if not s.eof and (self.engine.eof(cid) or st == _utp.RESET):
            s.eof = True
            if st == _utp.RESET and not s.connected.is_set():
                s.connected.set()
            s.reader.feed_eof()
            if s.sink_eof is not None:
                s.sink_eof()
        s.transport._push()

    def _flush(self) -> None:
        if self._sock is None:
            self.engine.outgoing()          # closed: drop
            return
        if self._pump.send() and not self._writing:
            self._writing = True
            self._loop.add_writer(self._sock.fileno(), self._on_writable)   # type: ignore[union-attr]

    def _on_writable(self) -> None:
        if self._sock is None or not self._pump.send():
            self._writing = False
            if self._sock is not None:
                self._loop.remove_writer(self._sock.fileno())   # type: ignore[union-attr]

    async def _tick_loop(self) -> None:
        try:
            while True:
                await asyncio.sleep(TICK)
                self.engine.tick(_now_us())
                for cid in list(self.streams):
                    self._service(cid)
                    if self.streams[cid].eof and self.streams[cid].transport.is_closing():
                        del self.streams[cid]
                self._flush()
        except asyncio.CancelledError:
            pass

    def stats(self, cid: int) -> dict:
        return self.engine.stats(cid)

    # ------------------------------------------------------------ api
    async def connect(self, host: str, port: int, timeout: float = 5.0
                      ) -> tuple[asyncio.StreamReader, asyncio.StreamWriter]:
        cid = self.engine.connect(_key((host, port)), _now_us())
        s = _Stream(self, cid, (host, port))
        self.streams[cid] = s
        self._flush()
        try:
            await asyncio.wait_for(s.connected.wait(), timeout)
        except asyncio.TimeoutError:
            s.transport.abort()
            raise UtpError(f"uTP connect to {host}:{port} timed out") from None
        if self.engine.state(cid) == _utp.RESET:
            raise UtpError(f"uTP connection to {host}:{port} reset")
        return s.reader, s.writer

    async def accept(self) -> tuple[asyncio.StreamReader, asyncio.StreamWriter, tuple[str, int]]:
        s = await self.accept_q.get()
        return s.reader, s.writer, s.transport.peer


async def serve(sock: UtpSocket, handler) -> asyncio.Task:
    """Run ``handler(reader, writer)`` for every accepted connection."""
    async def loop():
        with contextlib.suppress(asyncio.CancelledError):
            while True:
                r, w, _a = await sock.accept()
                asyncio.ensure_future(handler(r, w))
    return asyncio.ensure_future(loop())
