"""In-process HTTP origin (raw asyncio HTTP, ``rawserver``) with Range / HEAD / ETag /
Content-Disposition and fault injection — the stand-in for the media
servers the HTTP downloader talks to (the reference had no test origin).

``tls=(cert_pem, key_pem)`` serves https (OpenSSL via the relay module).
Fault knobs: ``ranges`` (advertise/honour Range), ``head`` (support HEAD),
``cut_after`` (drop the connection after N body bytes, once per request
count in ``cut_times``; ``cut_match`` limits it to one Range), ``fail_next`` (N × HTTP 500), ``rate`` (bytes/s cap),
``throttle`` (N × 429/503 with a ``Retry-After``), ``stall`` ((offset, seconds):
the next response goes silent for ``seconds`` after ``offset`` body bytes).
Without faults or a rate cap, GET bodies leave through ``sendfile`` from a
native thread (``SendfileResponse``) — blobs held in memory are mirrored to
a memfd once.
"""

from __future__ import annotations

import asyncio
import hashlib
import os
import re
from dataclasses import dataclass

from tritondl.utils import rawhttp
from . import rawserver as web


@dataclass
class Blob:
    data: bytes | None = None
    path: str | None = None
    disposition: str | None = None
    etag: str = ""

    def size(self) -> int:
        return len(self.data) if self.data is not None else os.path.getsize(self.path or "")

    def read(self, start: int, end: int) -> bytes:
        if self.data is not None:
            return self.data[start:end]
        with open(self.path or "", "rb") as f:
            f.seek(start)
            return f.read(end - start)

    def fd(self) -> int:
        """A read-only fd over the content for sendfile (memfd for in-memory blobs)."""
        fd = getattr(self, "_fd", None)
        if fd is None:
            if self.data is not None:
                fd = os.memfd_create("origin-blob", os.MFD_CLOEXEC)
                mv = memoryview(self.data)
                while mv:
                    mv = mv[os.write(fd, mv):]
            else:
                fd = os.open(self.path or "", os.O_RDONLY | os.O_CLOEXEC)
            self._fd = fd
        return fd


class Origin:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, *, tls: tuple[str, str] | None = None) -> None:
        """``tls``: (cert_pem, key_pem) to serve https."""
        self.host, self.port = host, port
        self.tls = tls
        self.blobs: dict[str, Blob] = {}
        self.ranges = True
        self.head = True
        self.cut_after: int | None = None
        self.cut_times = 0
        self.cut_match: str | None = None       # only cut requests whose Range header starts with this
        self.fail = 0
        self.throttle: tuple[int, int, str] | None = None   # (n, 429|503, Retry-After) for the next n GETs
        self.chunked = False                    # GET bodies with Transfer-Encoding: chunked (no ranges)
        self.rate: float | None = web.fake_stream_rate()     # bytes/s per response stream (None: uncapped)
        self.chunked_content_length: int | None = None   # chunked responses also claim this length
        self.latency = 0.0
        self.stall: tuple[int, float] | None = None   # (body offset, seconds): one mid-body silence
        self.requests: list[tuple[str, str, str]] = []
        self.redirects: dict[str, tuple[int, str]] = {}     # path -> (status, Location)
        self.basic_auth: dict[str, str] = {}    # path -> required "user:password" (401 otherwise)
        self.auth_seen: list[str] = []          # Authorization headers of the requests
        self._server: web.Server | None = None

    def add(self, path: str, data: bytes | None = None, *, file: str | None = None,
            disposition: str | None = None) -> str:
        etag = '"' + (hashlib.md5(data).hexdigest() if data is not None else f"f{os.path.getmtime(file or '')}") + '"'
        self.blobs[path] = Blob(data, file, disposition, etag)
        return self.url(path)

    def redirect(self, path: str, location: str, status: int = 302) -> str:
        """Answer ``path`` with a redirect to ``location`` (absolute or relative)."""
        self.redirects[path] = (status, location)
        return self.url(path)

    def url(self, path: str) -> str:
        return f"{'https' if self.tls else 'http'}://{self.host}:{self.port}{path}"

    async def start(self) -> "Origin":
        self._server = web.Server(self._handle, tls=self.tls)
        self.port = await self._server.start(self.host, self.port)
        return self

    async def stop(self) -> None:
        if self._server is not None:
            await self._server.stop()
            self._server = None

    async def _handle(self, request: web.Request) -> web.StreamResponse:
        self.requests.append((request.method, request.path, request.headers.get("Range", "")))
        if self.latency:
            await asyncio.sleep(self.latency)     # emulated one-way network delay per request
        if self.fail > 0:
            self.fail -= 1
            return web.Response(status=500, text="injected")
        if self.throttle and request.method == "GET":
            n, status, after = self.throttle
            self.throttle = (n - 1, status, after) if n > 1 else None
            return web.Response(status=status, text="slow down", headers={"Retry-After": str(after)})
        self.auth_seen.append(request.headers.get("Authorization", ""))
        need = self.basic_auth.get(request.path)
        if need is not None:
            import base64
            if request.headers.get("Authorization", "") != "Basic " + base64.b64encode(need.encode()).decode():
                return web.Response(status=401, text="unauthorized",
                                    headers={"WWW-Authenticate": 'Basic realm="media"'})
        rd = self.redirects.get(request.path)
        if rd is not None:
            return web.Response(status=rd[0], headers={"Location": rd[1]})
        blob = self.blobs.get(request.raw_path.split("?", 1)[0]) or self.blobs.get(request.path)
        if blob is None:
            return web.Response(status=404, text="not found")
        size = blob.size()
        hdrs = {"ETag": blob.etag, "Last-Modified": "Mon, 01 Jan 2024 00:00:00 GMT"}
        if self.ranges:
            hdrs["Accept-Ranges"] = "bytes"
        if blob.disposition:
            hdrs["Content-Disposition"] = blob.disposition
        if request.method == "HEAD":
            if not self.head:
                return web.Response(status=405)
            hdrs["Content-Length"] = str(size)
            return web.Response(status=200, headers=hdrs)
        if request.method != "GET":
            return web.Response(status=405)
        if self.chunked:
            return await self._chunked(request, blob, hdrs)
        start, end, status = 0, size, 200
        rng = request.headers.get("Range")
        if rng and self.ranges:
            ir = request.headers.get("If-Range")
            if ir is None or ir == blob.etag or ir == hdrs["Last-Modified"]:
                m = re.match(r"bytes=(\d+)-(\d*)$", rng)
                if not m:
                    return web.Response(status=416)
                start = int(m.group(1))
                end = int(m.group(2)) + 1 if m.group(2) else size
                end = min(end, size)
                if start >= size:
                    return web.Response(status=416, headers={"Content-Range": f"bytes */{size}"})
                status = 206
                hdrs["Content-Range"] = f"bytes {start}-{end - 1}/{size}"
        if self.cut_after is None and not self.rate and self.stall is None and rawhttp.relay_module() is not None:
            return web.SendfileResponse(status, hdrs, blob.fd(), start, end - start)
        hdrs["Content-Length"] = str(end - start)
        resp = web.StreamResponse(status=status, headers=hdrs)
        await resp.prepare(request)
        sent = 0
        step = 1 << 20
        pos = start
        while pos < end:
            n = min(step, end - pos)
            if self.cut_after is not None and self.cut_times > 0 and sent + n > self.cut_after and \
                    (self.cut_match is None or (rng or "").startswith(self.cut_match)):
                n = self.cut_after - sent
                if n > 0:
                    await resp.write(blob.read(pos, pos + n))
                self.cut_times -= 1
                request.transport.close()  # type: ignore[union-attr]
                return resp
            if self.stall is not None and sent <= self.stall[0] < sent + n:
                at, secs = self.stall
                self.stall = None
                k = at - sent
                if k:
                    await resp.write(blob.read(pos, pos + k))
                    pos, sent, n = pos + k, sent + k, n - k
                await asyncio.sleep(secs)       # the origin goes silent mid-body
            await resp.write(blob.read(pos, pos + n))
            pos += n
            sent += n
            if self.rate:
                await asyncio.sleep(n / self.rate)
        await resp.write_eof()
        return resp

    async def _chunked(self, request: web.Request, blob: Blob, hdrs: dict) -> web.StreamResponse:
        """The whole object with ``Transfer-Encoding: chunked`` (no length, no
        ranges — a dynamic origin): chunks of varying size, some with chunk
        extensions, and a trailer field; ``rate`` paces it."""
        import random
        hdrs = {k: v for k, v in hdrs.items() if k != "Accept-Ranges"}
        hdrs["Transfer-Encoding"] = "chunked"
        if self.chunked_content_length is not None:      # a broken server: both framings
            hdrs["Content-Length"] = str(self.chunked_content_length)
        resp = web.StreamResponse(status=200, headers=hdrs)
        await resp.prepare(request)
        rng = random.Random(len(self.requests))
        pos, size = 0, blob.size()
        while pos < size:
            n = min(size - pos, rng.choice((1, 7, 4096, 65536, 300_000)))
            ext = ";name=value" if rng.random() < 0.3 else ""
            await resp.write(f"{n:x}{ext}\r\n".encode() + blob.read(pos, pos + n) + b"\r\n")
            pos += n
            if self.rate:
                await asyncio.sleep(n / self.rate)
        await resp.write(b"0\r\nX-Checksum: none\r\n\r\n")
        return resp
