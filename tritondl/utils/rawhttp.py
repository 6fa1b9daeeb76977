"""Plain-HTTP/1.1 plumbing for the native data plane (``csrc/relay/``).

The control plane stays in asyncio: connect, write a request head, parse a
response head, read small bodies (S3 replies).  Large bodies never pass
through Python — the socket's fd is handed to ``_relay.recv_body`` /
``_relay.send_body``, which run in an executor thread with the GIL
released.  While a pump owns a socket, asyncio does not touch it.

Scope (everything else falls back to aiohttp in the callers): ``http://``
only (TLS stays in Python's ssl), identity transfer coding for downloads,
no redirects.  Idle keep-alive sockets are pooled per (host, port).
"""

from __future__ import annotations

import asyncio
import os
import socket
from dataclasses import dataclass, field

from multidict import CIMultiDict

from .log import log

_relay = None
_relay_checked = False

# opt-in event trace of the data plane (TRITONDL_TRACE=1): (event, monotonic time)
TRACE: list[tuple[str, float]] | None = [] if os.environ.get("TRITONDL_TRACE") else None


def trace(event: str) -> None:
    if TRACE is not None:
        import time
        TRACE.append((event, time.monotonic()))


def relay_module():
    """The ``_relay`` extension, or None (not built / disabled by
    ``TRITONDL_NATIVE_RELAY=0``); callers then use the aiohttp path."""
    global _relay, _relay_checked
    if not _relay_checked:
        _relay_checked = True
        if os.environ.get("TRITONDL_NATIVE_RELAY", "1").lower() in ("0", "off", "false", "no"):
            return None
        try:
            from .. import _relay as m  # type: ignore[attr-defined]
            _relay = m
        except ImportError as e:
            log.with_field("error", str(e)).warn("native relay extension missing; using the aiohttp data path "
                                                 "(run tools/build_native.py)")
    return _relay


class RawHTTPError(ConnectionError):
    pass


@dataclass
class Head:
    status: int
    reason: str
    headers: CIMultiDict
    leftover: bytes = b""          # body bytes that arrived with the head
    version: str = "HTTP/1.1"
    keep_alive: bool = True

    @property
    def content_length(self) -> int | None:
        v = self.headers.get("Content-Length")
        try:
            return int(v) if v is not None else None
        except ValueError:
            return None

    @property
    def chunked(self) -> bool:
        return "chunked" in self.headers.get("Transfer-Encoding", "").lower()


def split_host(hostport: str, default_port: int = 80) -> tuple[str, int]:
    if hostport.startswith("["):                       # [v6]:port
        h, _, rest = hostport[1:].partition("]")
        return h, int(rest[1:]) if rest.startswith(":") else default_port
    h, sep, p = hostport.rpartition(":")
    if sep and p.isdigit() and ":" not in h:
        return h, int(p)
    return hostport, default_port


@dataclass
class Pool:
    """Idle keep-alive sockets by (host, port)."""
    max_idle: int = 16
    idle: dict = field(default_factory=dict)

    async def connect(self, host: str, port: int, timeout: float = 30.0) -> tuple[socket.socket, bool]:
        """(socket, reused).  A pooled socket the peer has closed is dropped."""
        lst = self.idle.get((host, port))
        while lst:
            s = lst.pop()
            if _alive(s):
                return s, True
            s.close()
        loop = asyncio.get_running_loop()
        infos = await loop.getaddrinfo(host, port, type=socket.SOCK_STREAM)
        err: Exception | None = None
        for fam, typ, proto, _cn, addr in infos:
            s = socket.socket(fam, typ, proto)
            s.setblocking(False)
            try:
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                await asyncio.wait_for(loop.sock_connect(s, addr), timeout)
                return s, False
            except (OSError, asyncio.TimeoutError) as e:
                s.close()
                err = e
        raise RawHTTPError(f"connect {host}:{port}: {err}")

    def release(self, host: str, port: int, s: socket.socket) -> None:
        lst = self.idle.setdefault((host, port), [])
        if len(lst) >= self.max_idle:
            s.close()
        else:
            lst.append(s)

    def close(self) -> None:
        for lst in self.idle.values():
            for s in lst:
                s.close()
        self.idle.clear()


def _alive(s: socket.socket) -> bool:
    try:
        s.recv(1, socket.MSG_PEEK | socket.MSG_DONTWAIT)
        return False         # EOF, or stray bytes: not reusable either way
    except BlockingIOError:
        return True          # nothing pending, still open
    except OSError:
        return False


def request_head(method: str, target: str, headers: dict) -> bytes:
    lines = [f"{method} {target} HTTP/1.1"]
    lines += [f"{k}: {v}" for k, v in headers.items()]
    return ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1")


async def read_head(s: socket.socket, timeout: float, max_size: int = 64 << 10) -> Head:
    loop = asyncio.get_running_loop()
    buf = b""
    while True:
        i = buf.find(b"\r\n\r\n")
        if i >= 0:
            break
        if len(buf) > max_size:
            raise RawHTTPError("response head too large")
        try:
            d = await asyncio.wait_for(loop.sock_recv(s, 256 << 10), timeout)
        except asyncio.TimeoutError as e:
            raise RawHTTPError("timed out waiting for the response head") from e
        if not d:
            raise RawHTTPError("connection closed before the response head")
        buf += d
    lines = buf[:i].decode("latin-1").split("\r\n")
    ver, _, rest = lines[0].partition(" ")
    code, _, reason = rest.partition(" ")
    if not ver.startswith("HTTP/") or not code.isdigit():
        raise RawHTTPError(f"malformed status line {lines[0]!r}")
    hdrs: CIMultiDict = CIMultiDict()
    for ln in lines[1:]:
        k, sep, v = ln.partition(":")
        if sep:
            hdrs.add(k.strip(), v.strip())
    conn = hdrs.get("Connection", "").lower()
    keep = (ver == "HTTP/1.1" and conn != "close") or conn == "keep-alive"
    return Head(int(code), reason, hdrs, buf[i + 4:], ver, keep)


async def read_small_body(s: socket.socket, head: Head, timeout: float, limit: int = 16 << 20,
                          method: str = "GET") -> bytes:
    """Whole body of a small response (Content-Length, chunked, or until
    close).  Marks ``head.keep_alive`` False when the connection can't be
    reused."""
    loop = asyncio.get_running_loop()
    buf = bytearray(head.leftover)

    async def more() -> bool:
        try:
            d = await asyncio.wait_for(loop.sock_recv(s, 256 << 10), timeout)
        except asyncio.TimeoutError as e:
            raise RawHTTPError("timed out reading the response body") from e
        if not d:
            return False
        buf.extend(d)
        if len(buf) > limit:
            raise RawHTTPError("response body too large")
        return True

    if method == "HEAD" or head.status in (204, 304) or 100 <= head.status < 200:
        return b""
    if head.chunked:
        out = bytearray()
        pos = 0
        while True:
            while (j := buf.find(b"\r\n", pos)) < 0:
                if not await more():
                    raise RawHTTPError("connection closed inside a chunked body")
            n = int(bytes(buf[pos:j]).split(b";")[0] or b"0", 16)
            while len(buf) < j + 2 + n + 2:
                if not await more():
                    raise RawHTTPError("connection closed inside a chunked body")
            out += buf[j + 2:j + 2 + n]
            pos = j + 2 + n + 2
            if n == 0:
                # optional trailers end with an empty line; we just consumed the first CRLF
                return bytes(out)
    cl = head.content_length
    if cl is None:
        head.keep_alive = False
        while await more():
            pass
        return bytes(buf)
    while len(buf) < cl:
        if not await more():
            raise RawHTTPError("connection closed early")
    if len(buf) > cl:
        head.keep_alive = False
    return bytes(buf[:cl])
