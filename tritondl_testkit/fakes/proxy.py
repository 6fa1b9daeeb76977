"""In-process egress proxy for tests: an HTTP/1.1 forward proxy (absolute-form
requests and ``CONNECT`` tunnels) or a SOCKS5 proxy, with optional
credentials and an optional TLS listener (an ``https://`` proxy).

It stands in for the corporate / cluster egress proxy that the reference's
transports would go through via ``HTTP_PROXY`` / ``HTTPS_PROXY``
(grab's and minio-go's ``http.ProxyFromEnvironment``).  It counts what it
carries, so tests can prove a job went through it:

* ``requests``: the (method, absolute URL) of each forwarded request;
* ``connects``: the ``host:port`` of each tunnel;
* ``refused``: the number of 407 answers (or SOCKS authentication failures).

``hosts`` maps names to addresses.  Tests use names such as ``origin.test``
that only the proxy can resolve.  Go never proxies ``localhost`` or loopback
IPs, so the target cannot be named ``127.0.0.1``.  This also proves that the
client did not dial the target directly.
"""

from __future__ import annotations

import asyncio
import base64
import contextlib
import ssl
import struct
from urllib.parse import urlsplit

_HOP = ("proxy-authorization", "proxy-connection")


class FakeProxy:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, *, mode: str = "http",
                 auth: tuple[str, str] | None = None, hosts: dict[str, str] | None = None,
                 tls: tuple[str, str] | None = None) -> None:
        """``mode``: "http" (forward proxy + CONNECT) or "socks5".
        ``auth``: required (user, password).  ``tls``: (cert_pem, key_pem)
        to serve the proxy itself over TLS."""
        assert mode in ("http", "socks5")
        self.host, self.port, self.mode, self.auth = host, port, mode, auth
        self.hosts = dict(hosts or {})
        self.tls = tls
        self.requests: list[tuple[str, str]] = []
        self.connects: list[str] = []
        self.refused = 0
        self._server: asyncio.base_events.Server | None = None
        self._tasks: set[asyncio.Task] = set()
        self._writers: set[asyncio.StreamWriter] = set()

    @property
    def url(self) -> str:
        """The proxy URL without credentials (see :meth:`url_with`)."""
        scheme = "socks5" if self.mode == "socks5" else ("https" if self.tls else "http")
        return f"{scheme}://{self.host}:{self.port}"

    def url_with(self, user: str, password: str) -> str:
        scheme = "socks5" if self.mode == "socks5" else ("https" if self.tls else "http")
        return f"{scheme}://{user}:{password}@{self.host}:{self.port}"

    async def start(self) -> "FakeProxy":
        sctx = None
        if self.tls is not None:
            import os
            import tempfile
            sctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            with tempfile.TemporaryDirectory() as d:
                cf, kf = os.path.join(d, "c.pem"), os.path.join(d, "k.pem")
                with open(cf, "w") as f:
                    f.write(self.tls[0])
                with open(kf, "w") as f:
                    f.write(self.tls[1])
                sctx.load_cert_chain(cf, kf)
        self._server = await asyncio.start_server(self._serve, self.host, self.port, ssl=sctx)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    async def stop(self) -> None:
        if self._server is not None:
            self._server.close()
            for w in list(self._writers):
                w.close()
            for t in list(self._tasks):
                t.cancel()
            await asyncio.gather(*self._tasks, return_exceptions=True)
            with contextlib.suppress(Exception):
                await self._server.wait_closed()
            self._server = None

    # ------------------------------------------------------------ plumbing
    def _resolve(self, host: str) -> str:
        return self.hosts.get(host.lower(), host)

    def _authorized(self, value: str | None) -> bool:
        if self.auth is None:
            return True
        want = "Basic " + base64.b64encode(f"{self.auth[0]}:{self.auth[1]}".encode()).decode()
        return value == want

    async def _serve(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        task = asyncio.current_task()
        self._tasks.add(task)           # type: ignore[arg-type]
        self._writers.add(writer)
        try:
            if self.mode == "socks5":
                await self._socks(reader, writer)
            else:
                await self._http(reader, writer)
        except (ConnectionError, asyncio.IncompleteReadError, asyncio.LimitOverrunError, OSError, ValueError):
            pass
        finally:
            self._tasks.discard(task)   # type: ignore[arg-type]
            self._writers.discard(writer)
            writer.close()

    @staticmethod
    async def _pipe(r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
        try:
            while True:
                d = await r.read(1 << 20)
                if not d:
                    break
                w.write(d)
                await w.drain()
        except (ConnectionError, OSError):
            pass
        finally:
            with contextlib.suppress(Exception):
                if w.can_write_eof():
                    w.write_eof()

    # ------------------------------------------------------------ HTTP proxy
    @staticmethod
    def _parse_head(raw: bytes) -> tuple[str, str, list[tuple[str, str]]]:
        lines = raw.decode("latin-1").split("\r\n")
        method, target, _ver = lines[0].split(" ", 2)
        hdrs = []
        for ln in lines[1:]:
            if ":" in ln:
                k, v = ln.split(":", 1)
                hdrs.append((k.strip(), v.strip()))
        return method, target, hdrs

    @staticmethod
    def _get(hdrs, name: str) -> str | None:
        for k, v in hdrs:
            if k.lower() == name:
                return v
        return None

    @staticmethod
    async def _copy_body(r: asyncio.StreamReader, w: asyncio.StreamWriter, hdrs, *, until_eof: bool) -> bool:
        """Copy one message body; False when the connection must close after it."""
        te = (FakeProxy._get(hdrs, "transfer-encoding") or "").lower()
        if "chunked" in te:
            while True:
                line = await r.readuntil(b"\r\n")
                w.write(line)
                n = int(line.split(b";")[0].strip() or b"0", 16)
                if n == 0:
                    while True:                      # trailers, then the empty line
                        t = await r.readuntil(b"\r\n")
                        w.write(t)
                        if t == b"\r\n":
                            await w.drain()
                            return True
                left = n + 2
                while left:
                    d = await r.read(min(left, 1 << 20))
                    if not d:
                        raise ConnectionError("eof in chunked body")
                    w.write(d)
                    left -= len(d)
                await w.drain()
        cl = FakeProxy._get(hdrs, "content-length")
        if cl is not None:
            left = int(cl)
            while left:
                d = await r.read(min(left, 1 << 20))
                if not d:
                    raise ConnectionError("eof in body")
                w.write(d)
                left -= len(d)
                await w.drain()
            return True
        if until_eof:
            while True:
                d = await r.read(1 << 20)
                if not d:
                    break
                w.write(d)
                await w.drain()
            return False
        return True

    async def _http(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        upstream: dict[tuple[str, int], tuple[asyncio.StreamReader, asyncio.StreamWriter]] = {}
        try:
            while True:
                try:
                    raw = await reader.readuntil(b"\r\n\r\n")
                except asyncio.IncompleteReadError:
                    return
                method, target, hdrs = self._parse_head(raw[:-4])
                if not self._authorized(self._get(hdrs, "proxy-authorization")):
                    self.refused += 1
                    await self._copy_body(reader, _Null(), hdrs, until_eof=False)
                    writer.write(b"HTTP/1.1 407 Proxy Authentication Required\r\n"
                                 b"Proxy-Authenticate: Basic realm=\"fake\"\r\nContent-Length: 0\r\n\r\n")
                    await writer.drain()
                    continue
                if method == "CONNECT":
                    host, _, port = target.rpartition(":")
                    host = host.strip("[]")
                    self.connects.append(target)
                    try:
                        ur, uw = await asyncio.open_connection(self._resolve(host), int(port))
                    except OSError:
                        writer.write(b"HTTP/1.1 502 Bad Gateway\r\nContent-Length: 0\r\n\r\n")
                        await writer.drain()
                        return
                    writer.write(b"HTTP/1.1 200 Connection established\r\n\r\n")
                    await writer.drain()
                    try:
                        await asyncio.gather(self._pipe(reader, uw), self._pipe(ur, writer))
                    finally:
                        uw.close()
                    return
                u = urlsplit(target)
                if u.scheme != "http" or not u.hostname:
                    writer.write(b"HTTP/1.1 400 Bad Request\r\nContent-Length: 0\r\n\r\n")
                    await writer.drain()
                    return
                self.requests.append((method, target))
                key = (u.hostname, u.port or 80)
                if key not in upstream:
                    try:
                        upstream[key] = await asyncio.open_connection(self._resolve(key[0]), key[1])
                    except OSError:
                        writer.write(b"HTTP/1.1 502 Bad Gateway\r\nContent-Length: 0\r\n\r\n")
                        await writer.drain()
                        return
                ur, uw = upstream[key]
                path = (u.path or "/") + (f"?{u.query}" if u.query else "")
                out = [f"{method} {path} HTTP/1.1"] + [f"{k}: {v}" for k, v in hdrs if k.lower() not in _HOP]
                uw.write(("\r\n".join(out) + "\r\n\r\n").encode("latin-1"))
                await self._copy_body(reader, uw, hdrs, until_eof=False)
                await uw.drain()
                rraw = await ur.readuntil(b"\r\n\r\n")
                writer.write(rraw)
                status_line, rhdrs = self._parse_head_resp(rraw[:-4])
                status = int(status_line.split(" ")[1])
                keep = True
                if method != "HEAD" and status not in (204, 304) and status >= 200:
                    keep = await self._copy_body(ur, writer, rhdrs, until_eof=True)
                await writer.drain()
                conn_hdr = ((self._get(rhdrs, "connection") or "") + (self._get(hdrs, "connection") or "")).lower()
                if not keep or "close" in conn_hdr:
                    return
        finally:
            for _r, w in upstream.values():
                w.close()

    @staticmethod
    def _parse_head_resp(raw: bytes):
        lines = raw.decode("latin-1").split("\r\n")
        hdrs = []
        for ln in lines[1:]:
            if ":" in ln:
                k, v = ln.split(":", 1)
                hdrs.append((k.strip(), v.strip()))
        return lines[0], hdrs

    # ------------------------------------------------------------ SOCKS5
    async def _socks(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        ver, n = await reader.readexactly(2)
        methods = await reader.readexactly(n)
        if ver != 5:
            return
        want = 2 if self.auth is not None else 0
        if want not in methods:
            writer.write(b"\x05\xff")
            self.refused += 1
            await writer.drain()
            return
        writer.write(bytes([5, want]))
        await writer.drain()
        if want == 2:
            _v, ul = await reader.readexactly(2)
            user = (await reader.readexactly(ul)).decode()
            (pl,) = await reader.readexactly(1)
            pw = (await reader.readexactly(pl)).decode()
            ok = (user, pw) == self.auth
            writer.write(b"\x01\x00" if ok else b"\x01\x01")
            await writer.drain()
            if not ok:
                self.refused += 1
                return
        _v, cmd, _r, atyp = await reader.readexactly(4)
        if atyp == 1:
            import ipaddress
            host = str(ipaddress.IPv4Address(await reader.readexactly(4)))
        elif atyp == 4:
            import ipaddress
            host = str(ipaddress.IPv6Address(await reader.readexactly(16)))
        else:
            (ln,) = await reader.readexactly(1)
            host = (await reader.readexactly(ln)).decode()
        (port,) = struct.unpack(">H", await reader.readexactly(2))
        if cmd != 1:
            writer.write(b"\x05\x07\x00\x01" + b"\0" * 6)
            await writer.drain()
            return
        self.connects.append(f"{host}:{port}")
        try:
            ur, uw = await asyncio.open_connection(self._resolve(host), port)
        except OSError:
            writer.write(b"\x05\x05\x00\x01" + b"\0" * 6)
            await writer.drain()
            return
        writer.write(b"\x05\x00\x00\x01" + b"\0" * 6)
        await writer.drain()
        try:
            await asyncio.gather(self._pipe(reader, uw), self._pipe(ur, writer))
        finally:
            uw.close()


class _Null:
    """A writer that drops what it is given (body of a refused request)."""

    def write(self, _d: bytes) -> None:
        pass

    async def drain(self) -> None:
        pass
