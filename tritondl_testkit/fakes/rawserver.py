"""Minimal asyncio HTTP/1.1 server on raw sockets for the local fakes
(origin, S3).  It exposes the small slice of the ``aiohttp.web`` API the
fakes' handlers use (``Request.method/raw_path/path/query_string/headers/
read()/content.iter_chunked()/transport.close()``, ``Response``,
``StreamResponse``) plus two native hooks that keep bench-sized bodies out of
Python:

* ``Request.take_body()`` hands the socket (and the body bytes that arrived
  with the head) to a native pump, e.g. ``_relay.recv_verify_chunked``;
* ``SendfileResponse`` sends head + a file range with ``_relay.send_body``
  (sendfile from a native thread).

Keep-alive, Content-Length and chunked request bodies; one task per
connection; optional TLS (``Server(handler, tls=(cert_pem, key_pem))``) with
the relay module's OpenSSL streams, so the native hooks work over https too.
Not a general web server — a stand-in for MinIO / a media origin on the same
box.
"""

from __future__ import annotations

import asyncio
import contextlib
import socket
from urllib.parse import unquote

from multidict import CIMultiDict

from tritondl.utils import rawhttp

_REASONS = {200: "OK", 204: "No Content", 206: "Partial Content", 301: "Moved Permanently", 302: "Found",
            304: "Not Modified", 400: "Bad Request", 403: "Forbidden", 404: "Not Found",
            405: "Method Not Allowed", 409: "Conflict", 416: "Range Not Satisfiable",
            500: "Internal Server Error", 503: "Service Unavailable"}


class _Transport:
    def __init__(self, conn: "_Conn") -> None:
        self._conn = conn

    def close(self) -> None:
        self._conn.abort()


class _Content:
    def __init__(self, req: "Request") -> None:
        self._req = req

    async def iter_chunked(self, n: int):
        while True:
            d = await self._req._read_some(n)
            if not d:
                return
            yield d

    def at_eof(self) -> bool:
        return self._req._remaining == 0


class Request:
    def __init__(self, conn: "_Conn", method: str, target: str, version: str, headers: CIMultiDict,
                 leftover: bytes) -> None:
        self._conn = conn
        self.method = method
        self.raw_path = target
        self.path = unquote(target.split("?", 1)[0])
        self.query_string = target.split("?", 1)[1] if "?" in target else ""
        self.version = version
        self.headers = headers
        self.transport = _Transport(conn)
        self.content = _Content(self)
        self._buf = leftover
        te = headers.get("Transfer-Encoding", "").lower()
        self._chunked = "chunked" in te
        cl = headers.get("Content-Length")
        self._remaining = -1 if self._chunked else (int(cl) if cl else 0)
        self._taken = False
        self.transport_close_after = False   # reply, then drop the connection (body not fully read)
        self.idle_timeout: float | None = None   # body reads raise asyncio.TimeoutError after this silence

    @property
    def body_length(self) -> int | None:
        return None if self._chunked else self._remaining

    async def _recv(self, n: int) -> bytes:
        if self._buf:
            d, self._buf = self._buf[:n], self._buf[n:]
            return d
        if self.idle_timeout:
            return await asyncio.wait_for(self._conn.recv(n), self.idle_timeout)
        return await self._conn.recv(n)

    async def _read_some(self, n: int) -> bytes:
        if self._chunked:
            return await self._read_chunk_piece(n)
        if self._remaining <= 0:
            return b""
        d = await self._recv(min(n, self._remaining))
        if not d:
            raise ConnectionError("client closed inside the request body")
        self._remaining -= len(d)
        return d

    async def _read_chunk_piece(self, n: int) -> bytes:
        # de-chunk lazily: keep the state in _chunk_left
        left = getattr(self, "_chunk_left", 0)
        if left == 0:
            line = await self._readline()
            size = int(line.split(b";")[0].strip() or b"0", 16)
            if size == 0:
                while (await self._readline()) not in (b"", b"\r\n"):
                    pass
                self._chunked = False
                self._remaining = 0
                return b""
            left = size
        d = await self._recv(min(n, left))
        if not d:
            raise ConnectionError("client closed inside a chunked body")
        left -= len(d)
        if left == 0:
            await self._readline()          # CRLF after the chunk data
        self._chunk_left = left
        return d

    async def _readline(self) -> bytes:
        while b"\n" not in self._buf:
            d = await self._conn.recv(64 << 10)
            if not d:
                out, self._buf = self._buf, b""
                return out
            self._buf += d
        i = self._buf.index(b"\n")
        out, self._buf = self._buf[:i + 1], self._buf[i + 1:]
        return out

    async def read(self) -> bytes:
        parts = []
        while True:
            d = await self._read_some(1 << 20)
            if not d:
                return b"".join(parts)
            parts.append(d)

    def take_body(self):
        """Hand the raw body to a native pump: returns (native stream — a
        ``_relay.Sock`` or ``_relay.TlsConn`` —, bytes already buffered).  The
        caller must consume exactly ``body_length`` bytes."""
        assert not self._chunked, "take_body needs a Content-Length body"
        self._taken = True
        pre, self._buf = self._buf, b""
        n = min(len(pre), self._remaining)
        self._remaining = 0
        return self._conn.raw.native, pre[:n]


class Response:
    def __init__(self, *, status: int = 200, body: bytes | None = None, text: str | None = None,
                 headers: dict | None = None, content_type: str | None = None) -> None:
        self.status = status
        self.headers = dict(headers or {})
        if text is not None:
            body = text.encode()
            content_type = content_type or "text/plain; charset=utf-8"
        self.body = body or b""
        if content_type:
            self.headers.setdefault("Content-Type", content_type)


class SendfileResponse:
    """Head + ``length`` bytes of ``fd`` from ``offset``, sent by the native
    relay (sendfile) — the fake origin's bulk path."""

    def __init__(self, status: int, headers: dict, fd: int, offset: int, length: int) -> None:
        self.status, self.headers, self.fd, self.offset, self.length = status, dict(headers), fd, offset, length


class StreamResponse:
    def __init__(self, *, status: int = 200, headers: dict | None = None) -> None:
        self.status = status
        self.headers = dict(headers or {})
        self._conn: _Conn | None = None

    async def prepare(self, request: Request) -> None:
        self._conn = request._conn
        self._conn.streamed = self
        await self._conn.send(_head_bytes(self.status, self.headers, None))

    async def write(self, data: bytes) -> None:
        assert self._conn is not None
        await self._conn.send(data)

    async def write_eof(self) -> None:
        return None


def _head_bytes(status: int, headers: dict, length: int | None) -> bytes:
    h = dict(headers)
    if length is not None and not any(k.lower() == "content-length" for k in h):
        h["Content-Length"] = str(length)
    lines = [f"HTTP/1.1 {status} {_REASONS.get(status, 'Status')}"] + [f"{k}: {v}" for k, v in h.items()]
    return ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1")


class _Conn:
    def __init__(self, server: "Server", sock: socket.socket) -> None:
        self.server = server
        self.sock = sock
        self.loop = asyncio.get_running_loop()
        self.closed = False
        self.streamed: StreamResponse | None = None
        tls = None
        if server.tls is not None:
            tls = rawhttp.relay_module().TlsConn(server.tls, sock.fileno())
        self.raw = rawhttp.RawConn(sock, tls)

    async def recv(self, n: int) -> bytes:
        if self.closed:
            return b""
        try:
            return await self.raw.recv(n)
        except OSError:
            return b""

    async def send(self, data: bytes) -> None:
        if self.closed:
            raise ConnectionResetError("connection closed")
        await self.raw.sendall(data)

    def abort(self) -> None:
        if not self.closed:
            self.closed = True
            with contextlib.suppress(OSError):
                self.sock.shutdown(socket.SHUT_RDWR)

    async def serve(self) -> None:
        buf = b""
        rtt = self.server.rtt
        try:
            if rtt:
                await asyncio.sleep(rtt)                 # TCP handshake (SYN / SYN-ACK)
            if self.raw.tls is not None:
                await self.raw.handshake(30.0)
                if rtt:
                    await asyncio.sleep(rtt)             # TLS 1.3: one more round trip
            while not self.closed:
                while b"\r\n\r\n" not in buf:
                    d = await self.recv(256 << 10)
                    if not d:
                        return
                    buf += d
                    if len(buf) > (64 << 10) and b"\r\n\r\n" not in buf:
                        return
                i = buf.index(b"\r\n\r\n")
                lines = buf[:i].decode("latin-1").split("\r\n")
                buf = buf[i + 4:]
                try:
                    method, target, version = lines[0].split(" ", 2)
                except ValueError:
                    return
                hdrs: CIMultiDict = CIMultiDict()
                for ln in lines[1:]:
                    k, sep, v = ln.partition(":")
                    if sep:
                        hdrs.add(k.strip(), v.strip())
                req = Request(self, method, target, version, hdrs, buf)
                buf = b""
                self.streamed = None
                if rtt:
                    await asyncio.sleep(rtt)             # request -> response round trip
                resp = await self.server.handler(req)
                if self.closed:
                    return
                # drain what the handler left of the body (keeps the connection in sync),
                # unless the connection is dropped after this reply anyway
                if not req._taken and not req.transport_close_after:
                    while await req._read_some(1 << 20):
                        pass
                buf = req._buf
                if self.streamed is None:
                    if isinstance(resp, SendfileResponse):
                        await self._sendfile(resp)
                    else:
                        body = b"" if method == "HEAD" else resp.body
                        length = None if (method == "HEAD" and "Content-Length" in resp.headers) else len(resp.body)
                        await self.send(_head_bytes(resp.status, resp.headers, length) + body)
                conn_hdr = hdrs.get("Connection", "").lower()
                if req.transport_close_after or conn_hdr == "close" or (version == "HTTP/1.0" and conn_hdr != "keep-alive"):
                    return
        except (ConnectionError, OSError, asyncio.TimeoutError):
            return
        finally:
            self.closed = True
            self.raw.close()

    async def _sendfile(self, resp: SendfileResponse) -> None:
        head = _head_bytes(resp.status, resp.headers, resp.length)
        relay = rawhttp.relay_module()
        if relay is None:
            assert self.raw.tls is None, "TLS needs the relay extension"
            await self.send(head)
            await self.loop.sock_sendfile(self.sock, _FdFile(resp.fd), resp.offset, resp.length)
            return
        if self.raw.tls is None:
            # the head leaves now, from the loop (one non-blocking send), so the
            # client parses it while the pump thread is still being woken
            await self.send(head)
            head = b""
        _sent, _sig, err = await rawhttp.run_pump(self.raw, relay.send_body, head, resp.fd, resp.offset,
                                                  resp.length, None, 0)
        if err:
            raise ConnectionResetError(err)


class _FdFile:
    """File-object shim over a raw fd for ``loop.sock_sendfile``."""

    def __init__(self, fd: int) -> None:
        self._fd = fd

    def fileno(self) -> int:
        return self._fd

    def seek(self, pos: int, whence: int = 0) -> int:
        import os
        return os.lseek(self._fd, pos, whence)

    def tell(self) -> int:
        import os
        return os.lseek(self._fd, 0, 1)

    def read(self, n: int = -1) -> bytes:
        import os
        return os.read(self._fd, n if n >= 0 else 1 << 30)


def fake_rtt() -> float:
    """Emulated network round trip of the fakes, seconds (``TRITONDL_FAKE_RTT_MS``;
    bench.py ``--rtt-ms``).  A latency model, not a bandwidth one: every new
    connection, TLS handshake and request/response exchange waits one RTT
    (the broker delays every frame it sends by one RTT); bytes then flow at
    loopback speed."""
    import os
    try:
        return max(0.0, float(os.environ.get("TRITONDL_FAKE_RTT_MS", "0") or 0) / 1000.0)
    except ValueError:
        return 0.0


def fake_stream_rate() -> float | None:
    """Per-stream bandwidth cap of the fake origin / S3, bytes/s
    (``TRITONDL_FAKE_STREAM_MBPS``, Mbit/s; bench.py ``--stream-mbps``): one
    TCP stream's window / RTT on a real path, which is what parallel Range
    streams and parallel multipart parts exist to beat.  None = uncapped."""
    import os
    try:
        v = float(os.environ.get("TRITONDL_FAKE_STREAM_MBPS", "0") or 0)
    except ValueError:
        return None
    return v * 1e6 / 8 if v > 0 else None


class Server:
    def __init__(self, handler, tls: tuple[str, str] | None = None, rtt: float | None = None) -> None:
        """``tls``: (cert_pem, key_pem) to serve https.  ``rtt``: emulated round
        trip (s; default :func:`fake_rtt`)."""
        self.handler = handler
        self.rtt = fake_rtt() if rtt is None else rtt
        self.tls = rawhttp.relay_module().TlsContext.server(*tls) if tls is not None else None
        self._srv: asyncio.base_events.Server | None = None
        self._conns: set[asyncio.Task] = set()
        self.port = 0

    async def start(self, host: str, port: int) -> int:
        loop = asyncio.get_running_loop()
        lsock = socket.socket(socket.AF_INET6 if ":" in host else socket.AF_INET, socket.SOCK_STREAM)
        lsock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        lsock.bind((host, port))
        lsock.listen(256)
        lsock.setblocking(False)
        self._lsock = lsock
        self.port = lsock.getsockname()[1]
        self._accept_task = asyncio.ensure_future(self._accept_loop(loop))
        return self.port

    async def _accept_loop(self, loop) -> None:
        while True:
            try:
                s, _addr = await loop.sock_accept(self._lsock)
            except (OSError, asyncio.CancelledError):
                return
            s.setblocking(False)
            with contextlib.suppress(OSError):
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            t = asyncio.ensure_future(_Conn(self, s).serve())
            self._conns.add(t)
            t.add_done_callback(self._conns.discard)

    async def stop(self) -> None:
        self._accept_task.cancel()
        with contextlib.suppress(BaseException):
            await self._accept_task
        self._lsock.close()
        for t in list(self._conns):
            t.cancel()
        for t in list(self._conns):
            with contextlib.suppress(BaseException):
                await t
