"""HTTPS origin that speaks HTTP/2 (ALPN ``h2``): the stand-in for a CDN in
the HTTP/2 tests and A/B (:mod:`tritondl.fetch.h2`).

It serves blobs with Range / ETag / Last-Modified / Content-Disposition like
:class:`~tritondl_testkit.fakes.origin.Origin`, over one TLS connection per
client with any number of concurrent streams.  It behaves like a real
server where a client can go wrong: response headers are HPACK-coded with
Huffman strings and incremental indexing (the client's dynamic table must
follow), DATA frames respect the client's flow-control windows and its
SETTINGS_MAX_FRAME_SIZE, and PING / RST_STREAM / GOAWAY are honoured.
``TRITONDL_FAKE_RTT_MS`` delays a new connection by two round trips and
each response head by one, as the HTTP/1.1 fakes do.
Fault and shaping knobs: ``stream_rate`` (bytes/s per stream),
``conn_rate`` (bytes/s per connection: one TCP window over a WAN path),
``pad`` (pad every DATA frame), ``frame_size`` (largest DATA frame),
``max_streams`` (SETTINGS_MAX_CONCURRENT_
STREAMS), ``goaway_after`` (GOAWAY after that many streams), ``stall`` ((offset,
seconds): one stream goes silent mid-body), ``alpn``
(offer only ``http/1.1`` to test the fallback); ``redirects`` maps a path
to the Location of a 301.
"""

from __future__ import annotations

import asyncio
import hashlib
import os
import re
import ssl
import struct
import tempfile
import time

from tritondl.fetch.h2 import (ACK, CONTINUATION, DATA, END_HEADERS, END_STREAM, GOAWAY, HEADERS, PADDED,
                               PING, PREFACE, RST_STREAM, S_INITIAL_WINDOW_SIZE, S_MAX_CONCURRENT_STREAMS,
                               S_MAX_FRAME_SIZE, SETTINGS, WINDOW_UPDATE, frame)
from tritondl.utils.hpack import Decoder, Encoder


class _Conn:
    def __init__(self, srv: "H2Origin", r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
        self.srv, self.r, self.w = srv, r, w
        self.enc = Encoder(huffman=True, index=True)
        self.dec = Decoder()
        self.lock = asyncio.Lock()                 # HPACK state and frame order: one writer at a time
        self.conn_window = 65535
        self.init_window = 65535
        self.max_frame = 16384
        self.windows: dict[int, int] = {}
        self.tasks: dict[int, asyncio.Task] = {}
        self.credit = asyncio.Event()
        self.streams = 0
        self.sent_at = time.monotonic()
        self.sent = 0

    async def run(self) -> None:
        if await self.r.readexactly(len(PREFACE)) != PREFACE:
            return
        self.w.write(frame(SETTINGS, 0, 0, struct.pack(">HI", S_MAX_CONCURRENT_STREAMS, self.srv.max_streams)))
        hblock: bytearray | None = None
        hsid = 0
        try:
            while True:
                head = await self.r.readexactly(9)
                ln = (head[0] << 16) | (head[1] << 8) | head[2]
                ftype, flags = head[3], head[4]
                sid = struct.unpack(">I", head[5:9])[0] & 0x7FFFFFFF
                payload = await self.r.readexactly(ln) if ln else b""
                if ftype == SETTINGS and not flags & ACK:
                    for k in range(0, len(payload) - 5, 6):
                        key, val = struct.unpack(">HI", payload[k:k + 6])
                        if key == S_INITIAL_WINDOW_SIZE:
                            for s in self.windows:
                                self.windows[s] += val - self.init_window
                            self.init_window = val
                        elif key == S_MAX_FRAME_SIZE:
                            self.max_frame = val
                    self.w.write(frame(SETTINGS, ACK, 0))
                    self.credit.set()
                elif ftype == WINDOW_UPDATE:
                    inc = struct.unpack(">I", payload)[0] & 0x7FFFFFFF
                    if sid == 0:
                        self.conn_window += inc
                    elif sid in self.windows:
                        self.windows[sid] += inc
                    self.credit.set()
                elif ftype in (HEADERS, CONTINUATION):
                    hblock = bytearray(payload) if ftype == HEADERS else hblock + payload   # type: ignore[operator]
                    hsid = sid if ftype == HEADERS else hsid
                    if flags & END_HEADERS:
                        fields = dict(self.dec.decode(bytes(hblock)))
                        hblock = None
                        self.streams += 1
                        self.srv.streams += 1
                        if self.srv.goaway_after and self.streams > self.srv.goaway_after:
                            async with self.lock:
                                self.w.write(frame(GOAWAY, 0, 0, struct.pack(">II", hsid - 2, 0)))
                            continue
                        if len(self.tasks) >= self.srv.max_streams:
                            # RFC 9113 5.1.2: over SETTINGS_MAX_CONCURRENT_STREAMS: refuse, retryable
                            async with self.lock:
                                self.w.write(frame(RST_STREAM, 0, hsid, struct.pack(">I", 7)))
                            self.srv.refused += 1
                            continue
                        self.windows[hsid] = self.init_window
                        self.tasks[hsid] = asyncio.ensure_future(self._serve(hsid, fields))
                elif ftype == RST_STREAM:
                    t = self.tasks.pop(sid, None)
                    if t is not None:
                        t.cancel()
                    self.srv.resets += 1
                elif ftype == PING and not flags & ACK:
                    self.w.write(frame(PING, ACK, 0, payload))
                elif ftype == GOAWAY:
                    return
        except (asyncio.IncompleteReadError, ConnectionError, OSError):
            pass
        finally:
            for t in self.tasks.values():
                t.cancel()
            self.w.close()

    async def _serve(self, sid: int, req: dict) -> None:
        try:
            await self._respond(sid, req)
        finally:                                    # every way out frees the stream's slot
            self.windows.pop(sid, None)
            self.tasks.pop(sid, None)

    async def _respond(self, sid: int, req: dict) -> None:
        srv = self.srv
        if srv.rtt:
            await asyncio.sleep(srv.rtt)              # emulated round trip: request out, head back
        path = req.get(b":path", b"/").decode()
        rng = req.get(b"range", b"").decode()
        srv.requests.append(("GET", path, rng))
        loc = srv.redirects.get(path)
        if loc is not None:
            await self._head(sid, [(b":status", b"301"), (b"location", loc.encode())], end=True)
            return
        blob = srv.lookup(path.split("?", 1)[0])
        if blob is None:
            await self._head(sid, [(b":status", b"404")], end=True)
            return
        data, etag, disposition = blob
        size = len(data)
        start, end, status = 0, size, 200
        hdrs = [(b"accept-ranges", b"bytes"), (b"etag", etag.encode()),
                (b"last-modified", b"Mon, 01 Jan 2024 00:00:00 GMT"), (b"server", b"tritondl-fake-h2")]
        ir = req.get(b"if-range")
        m = re.match(r"bytes=(\d+)-(\d*)$", rng) if rng else None
        if m and (ir is None or ir.decode() in (etag, "Mon, 01 Jan 2024 00:00:00 GMT")):
            start = int(m.group(1))
            end = min(size, int(m.group(2)) + 1) if m.group(2) else size
            if start >= size:
                await self._head(sid, [(b":status", b"416"), (b"content-range", f"bytes */{size}".encode())],
                                 end=True)
                return
            status = 206
            hdrs.append((b"content-range", f"bytes {start}-{end - 1}/{size}".encode()))
        if disposition:
            hdrs.append((b"content-disposition", disposition.encode()))
        hdrs.append((b"content-length", str(end - start).encode()))
        await self._head(sid, [(b":status", str(status).encode())] + hdrs, end=end == start)
        pos = start
        t0 = time.monotonic()
        while pos < end:
            while self.conn_window <= 0 or self.windows.get(sid, 0) <= 0:
                self.credit.clear()
                await self.credit.wait()
            n = min(end - pos, min(self.max_frame, srv.frame_size) - (8 if srv.pad else 0), self.conn_window,
                    self.windows[sid])
            if srv.stall is not None and pos - start <= srv.stall[0] < pos - start + n:
                at, secs = srv.stall
                if at > pos - start:
                    n = at - (pos - start)
                else:
                    srv.stall = None
                    await asyncio.sleep(secs)     # this stream goes silent mid-body
            body = data[pos:pos + n]
            flags = END_STREAM if pos + n >= end else 0
            if srv.pad:
                payload = bytes([7]) + body + b"\0" * 7
                flags |= PADDED
            else:
                payload = body
            async with self.lock:
                self.w.write(frame(DATA, flags, sid, payload))
                self.conn_window -= len(payload)
                self.windows[sid] -= len(payload)
                await self.w.drain()
            pos += n
            srv.bytes_sent += n
            if srv.stream_rate:
                wait = t0 + (pos - start) / srv.stream_rate - time.monotonic()
                if wait > 0:
                    await asyncio.sleep(wait)
            if srv.conn_rate:
                self.sent += n
                wait = self.sent_at + self.sent / srv.conn_rate - time.monotonic()
                if wait > 0:
                    await asyncio.sleep(wait)

    async def _head(self, sid: int, fields: list, end: bool) -> None:
        async with self.lock:
            block = self.enc.encode(fields)
            mx = self.max_frame
            first, rest = block[:mx], block[mx:]
            out = [frame(HEADERS, (END_STREAM if end else 0) | (0 if rest else END_HEADERS), sid, first)]
            while rest:
                part, rest = rest[:mx], rest[mx:]
                out.append(frame(CONTINUATION, 0 if rest else END_HEADERS, sid, part))
            self.w.write(b"".join(out))
            await self.w.drain()


class H2Origin:
    def __init__(self, host: str = "127.0.0.1", *, alpn: tuple[str, ...] = ("h2", "http/1.1"), port: int = 0,
                 cert_pem: str = "", key_pem: str = "") -> None:
        """``cert_pem`` / ``key_pem``: serve this certificate (else a throwaway
        test PKI whose CA is ``ca_pem`` / ``ca_file``)."""
        from tritondl.utils import rawhttp
        self.host, self.port = host, port
        self.alpn = alpn
        self.blobs: dict[str, tuple[bytes, str, str]] = {}
        self.redirects: dict[str, str] = {}          # path -> Location of a 301
        self.requests: list[tuple[str, str, str]] = []
        self.connections = 0
        self.streams = 0
        self.resets = 0
        self.refused = 0                             # streams refused over max_streams (RST REFUSED_STREAM)
        self.frame_size = 1 << 20                    # largest DATA frame sent (nginx sends ~16 KiB ones)
        from .rawserver import fake_rtt
        self.rtt = fake_rtt()                        # TRITONDL_FAKE_RTT_MS: connection + TLS + each request
        self.bytes_sent = 0
        self.stream_rate: float | None = None
        self.conn_rate: float | None = None
        self.pad = False
        self.max_streams = 100
        self.goaway_after = 0
        self.stall: tuple[int, float] | None = None   # (body offset, seconds): the next stream to reach it goes silent
        if cert_pem and key_pem:
            ca, cert, key = "", cert_pem, key_pem
        else:
            ca, cert, key = rawhttp.relay_module().make_test_pki([host, "localhost"])
        self._dir = tempfile.mkdtemp(prefix="tdl-h2-")
        self.ca_file = os.path.join(self._dir, "ca.pem")
        for name, pem in (("ca.pem", ca), ("cert.pem", cert), ("key.pem", key)):
            with open(os.path.join(self._dir, name), "w") as f:
                f.write(pem)
        self.ca_pem = ca
        self._server: asyncio.AbstractServer | None = None

    def lookup(self, path: str):
        """(data, etag, disposition) served at ``path``, or None (404)."""
        return self.blobs.get(path)

    def add(self, path: str, data: bytes, disposition: str = "") -> str:
        self.blobs[path] = (data, '"' + hashlib.md5(data).hexdigest() + '"', disposition)
        return self.url(path)

    def url(self, path: str) -> str:
        return f"https://{self.host}:{self.port}{path}"

    async def start(self) -> "H2Origin":
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(os.path.join(self._dir, "cert.pem"), os.path.join(self._dir, "key.pem"))
        ctx.set_alpn_protocols(list(self.alpn))

        async def handle(r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
            self.connections += 1
            if self.rtt:
                await asyncio.sleep(2 * self.rtt)     # TCP connect + TLS handshake round trips
            sslobj = w.get_extra_info("ssl_object")
            if sslobj is None or sslobj.selected_alpn_protocol() != "h2":
                w.close()                      # this fake serves HTTP/2 only
                return
            await _Conn(self, r, w).run()

        self._server = await asyncio.start_server(handle, self.host, self.port, ssl=ctx)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    async def stop(self) -> None:
        if self._server is not None:
            self._server.close()
            await self._server.wait_closed()
            self._server = None
