"""HTTP(S) downloader — reference component C6
(``internal/downloader/http/http.go``, built on cavaliercoder/grab).

Registration: name ``http``, protocols ``http``/``https``, no extensions
(``http.go:25-33``).  Like grab: a probe discovers size, range support and
the file name (Content-Disposition, else the URL path's base name); an
existing complete file is not fetched again; an interrupted download resumes
with HTTP Range requests.  grab probes with HEAD; by default the probe here
is the first data request itself (``GET Range: bytes=0-``, kept open as the
first segment's stream), one round trip fewer per job (``probe="head"``
restores grab's order).  Progress is reported every
``progress_interval`` seconds and a final 100 (``http.go:45-67``).

Beyond the reference:

* errors are surfaced (B1: ``resp.Err()`` was never checked);
* progress is 0..100 (B2);
* the file is written as ``<name>.part`` + ``<name>.part.meta`` and renamed
  on completion, so a crash never leaves a truncated file that looks done,
  and ``If-Range`` guards against resuming onto a changed origin object;
* large files are fetched as ``segments`` concurrent Range streams written
  with ``pwrite`` from worker threads (grab used one stream) — contiguous
  slices, or with ``stripe_bytes`` in-order stripes pulled by ``segments``
  stream workers so the upload-visible watermark advances steadily; with
  ``probe_bytes`` (opt-in: ``TRITONDL_HTTP_PROBE_BYTES``) the
  probe is ``GET bytes=0-(probe_bytes-1)`` and the rest of a bigger file is
  requested at once as parallel Range streams, so mid-size files are
  segmented too and no half-read probe connection is dropped;
* ``http`` and ``https`` bodies never enter Python: after the head is
  parsed the connection (a plain socket, or an OpenSSL TLS session driven by
  the relay module) goes to the native receive pump (``csrc/relay``, GIL
  released), which writes the file and publishes progress on a native
  ``Flow`` that the S3 send pump follows; redirects are followed natively
  (later Range requests go straight to the final URL); chunked bodies are
  decoded by the pump (one GET, connection reused), content-coded bodies are
  stored as sent, as the aiohttp path does; aiohttp remains for odd 3xx
  replies, TLS through an https proxy, and builds without the relay module;
* the egress proxy of ``HTTP_PROXY`` / ``HTTPS_PROXY`` / ``NO_PROXY`` is used
  with Go's rules (:mod:`tritondl.utils.proxy`), as grab's transport did;
* the file's mtime is set from ``Last-Modified``, as grab does;
* when one segment fails, its siblings are cancelled and their pumps
  stopped and awaited before the file or any socket is closed (no write
  through a recycled fd number);
* with ``http2`` (``TRITONDL_HTTP2=1``) an https origin is first offered
  HTTP/2 in the TLS handshake, as Go's transport under grab did: if it
  accepts, the probe and every Range segment are streams of one connection
  (:mod:`tritondl.fetch.h2`); an origin that keeps to HTTP/1.1 is
  remembered and served by the paths above.
"""

from __future__ import annotations

import asyncio
import json
import os
import re
import time
from dataclasses import dataclass
from email.message import Message as _EmailMsg
from urllib.parse import unquote, urlparse

import aiohttp
from yarl import URL

from ..utils import proxy as _proxy
from ..utils import rawhttp, spares
from ..utils.dial import FALLBACK_DELAY, socket_factory
from ..utils.disk import DiskSpaceError, check_space
from ..utils.log import log
from . import h2 as _h2
from .registry import ClientRegister, ProgressSink


class HTTPDownloadError(Exception):
    pass


class _FatalHTTPError(HTTPDownloadError):
    pass


class _RetryLater(HTTPDownloadError):
    """429 / 503 with a ``Retry-After`` the job can wait out in place."""

    def __init__(self, msg: str, after: float) -> None:
        super().__init__(msg)
        self.after = after


def retry_after(r) -> float | None:
    """Seconds a 429 / 503 response asks the client to wait (``Retry-After``:
    delta-seconds or an HTTP-date, RFC 9110 §10.2.3), else None."""
    if r.status not in (429, 503):
        return None
    v = (r.headers.get("Retry-After") or "").strip()
    if not v:
        return None
    if v.isdigit():
        return float(v)
    try:
        from email.utils import parsedate_to_datetime
        import datetime
        when = parsedate_to_datetime(v)
        return max(0.0, (when - datetime.datetime.now(datetime.timezone.utc)).total_seconds())
    except (TypeError, ValueError, IndexError):
        return None


class _H2Content:
    def __init__(self, st: "_h2.H2Stream", read_timeout: float) -> None:
        self._st = st
        self._timeout = read_timeout

    async def iter_chunked(self, n: int):
        """Body chunks; a stream silent for the read timeout fails like an
        HTTP/1.1 body would (a retryable connection error)."""
        while True:
            try:
                b = await asyncio.wait_for(self._st.read(n), self._timeout)
            except asyncio.TimeoutError:
                self._st.cancel()
                raise aiohttp.ServerTimeoutError(
                    f"HTTP/2 stream {self._st.id}: no body bytes for {self._timeout:g} s") from None
            if not b:
                return
            yield b

    def at_eof(self) -> bool:
        return self._st.at_eof()


class _H2Response:
    """The bits of an aiohttp response this module uses, over one HTTP/2
    stream (its body is read by :meth:`HTTPDownloader._consume`)."""

    def __init__(self, st: "_h2.H2Stream", url: str, read_timeout: float = 120.0) -> None:
        self.st = st
        self.status = st.status
        self.headers = st.headers
        self.url = URL(url)
        self.content = _H2Content(st, read_timeout)

    def release(self) -> None:
        self.st.cancel()            # a no-op once the body has ended

    def close(self) -> None:
        self.st.cancel()


class _RawResponse:
    """The bits of an aiohttp response this module uses, over a raw
    connection (plain or TLS) whose body the native pump reads."""

    def __init__(self, pool: rawhttp.Pool, host: str, port: int, conn: rawhttp.RawConn, head: rawhttp.Head,
                 url: str) -> None:
        self.pool, self.host, self.port, self.sock, self.head = pool, host, port, conn, head
        self.status = head.status
        self.headers = head.headers
        self.url = URL(url)
        self.leftover = head.leftover
        self.complete = False          # body read to its end (connection reusable)

    def release(self) -> None:
        if self.sock is None:
            return
        if self.complete and self.head.keep_alive:
            self.pool.release(self.host, self.port, self.sock)
        else:
            self.sock.close()
        self.sock = None

    def close(self) -> None:
        if self.sock is not None:
            self.sock.close()
            self.sock = None


@dataclass
class _Probe:
    size: int | None
    ranges: bool
    etag: str
    last_modified: str
    filename: str
    status: int
    first_end: int | None = None     # end (exclusive) of the GET probe's 206 body
    final_url: str = ""              # after redirects: later Range requests go straight there


def filename_from_disposition(cd: str | None) -> str:
    if not cd:
        return ""
    m = _EmailMsg()
    m["content-disposition"] = cd
    name = m.get_filename() or ""
    if not name:
        mm = re.search(r"filename\*?=([^;]+)", cd)
        name = mm.group(1).strip().strip('"') if mm else ""
    return _safe_name(name)


# longest name the work dir can hold with the ``.part.meta.tmp`` sidecar suffix
_NAME_MAX = 255 - len(".part.meta.tmp")
_CONTROLS = re.compile(r"[\x00-\x1f\x7f]")


def _safe_name(name: str) -> str:
    """The last path component of a server- or URL-supplied name, "" when
    there is none.  C0 controls and DEL (NUL cannot be in a file name) become
    ``_``; text that is not valid UTF-8 becomes ``?``; a name longer than the
    file system allows next to its sidecars is cut in its stem on a character
    boundary, keeping the extension the media filter selects on.  The
    reference takes ``filepath.Base`` and fails on the rest."""
    name = name.replace("\\", "/").split("/")[-1]
    if name in ("", ".", ".."):
        return ""
    name = _CONTROLS.sub("_", name).encode("utf-8", "replace").decode("utf-8")
    if len(name.encode()) > _NAME_MAX:
        stem, dot, ext = name.rpartition(".")
        if not (dot and stem and len(ext.encode()) < 32):
            stem, dot, ext = name, "", ""
        keep = _NAME_MAX - len((dot + ext).encode())
        name = stem.encode()[:keep].decode("utf-8", "ignore") + dot + ext
    return name


def filename_from_url(url: str) -> str:
    return _safe_name(unquote(urlparse(url).path))


def _segments_ok(segs, size: int | None) -> bool:
    """A resume plan read back from ``.part.meta`` is used only if its
    ``[start, end, done]`` segments tile ``[0, size)`` in order with
    ``0 <= done <= end - start`` (one open-ended ``[0, -1, done]`` segment
    when the size is unknown); anything else restarts the download rather
    than leaving unwritten holes in the file."""
    if not isinstance(segs, list) or not segs:
        return False
    if not all(isinstance(sg, list) and len(sg) == 3 and all(type(v) is int for v in sg) for sg in segs):
        return False
    if size is None:
        return len(segs) == 1 and segs[0][0] == 0 and segs[0][1] == -1 and segs[0][2] >= 0
    at = 0
    for a, b, d in segs:
        if a != at or b < a or not 0 <= d <= b - a:
            return False
        at = b
    return at == size


class HTTPDownloader:
    def __init__(self, *, progress_interval: float = 1.0, segments: int = 4, segment_threshold: int = 64 << 20,
                 chunk: int = 1 << 20, write_block: int = 4 << 20, session: aiohttp.ClientSession | None = None,
                 headers: dict | None = None, max_retries: int = 5, probe: str = "get",
                 native: bool = True, read_timeout: float = 120.0, probe_bytes: int = 0,
                 ca_pem: str = "", ca_file: str = "", stripe_bytes: int = 0, max_redirects: int = 10,
                 disk_reserve: int = 0, proxies: "_proxy.ProxyConfig | None" = None, http2: bool = False,
                 h2_native: bool = True, h2_idle_s: float = 90.0, h2_conns: int = 4) -> None:
        self.progress_interval = progress_interval
        # offer HTTP/2 to https origins (ALPN), as Go's transport under grab did
        self.http2 = http2
        # HTTP/2 over the relay's TLS with a native session pump (False: asyncio's TLS, bodies in Python)
        self.h2_native = h2_native
        # an HTTP/2 connection with no stream for this long is closed (Go's IdleConnTimeout): a worker
        # that meets thousands of origins keeps a socket (and, native, a pump thread) only for live ones
        self.h2_idle_s = h2_idle_s
        # HTTP/2 connections per origin: a stream goes to the least busy one, and a new one opens
        # while every open one carries a stream (1 = one connection per origin, as Go's transport)
        self.h2_conns = max(1, h2_conns)
        self._h2closing: set[asyncio.Task] = set()
        self._h2conns: dict[tuple[str, int], list["_h2.H2Connection"]] = {}
        self._h2locks: dict[tuple[str, int], asyncio.Lock] = {}
        self._h1_only: dict[tuple[str, int], float] = {}     # origins that answered ALPN with http/1.1
        self.h2_streams = 0
        # egress proxy (HTTP_PROXY / HTTPS_PROXY / NO_PROXY, Go semantics); None = the environment
        self.proxies = proxies
        self.disk_reserve = disk_reserve            # bytes to keep free (utils.disk preflight)
        self.max_redirects = max_redirects          # Go's http.Client default (grab uses it)
        # >0: instead of `segments` contiguous slices, the file is cut into stripes of
        # this size handed out IN ORDER to `segments` stream workers (each reuses its
        # keep-alive connection).  All streams then advance through the file together,
        # so the contiguous-bytes watermark -- which the streamed S3 upload follows --
        # moves steadily instead of jumping when the last slice completes.  Opt-in
        # (TRITONDL_HTTP_STRIPE_BYTES): on the 10 MiB headline job every extra Range
        # request cost more than the smoother watermark won (http 219-225 vs 298 jobs/s,
        # https 147-163 vs 175; profiles/r02_stripe_ab)
        self.stripe_bytes = max(0, stripe_bytes)
        # >0: the GET probe asks for bytes=0-(probe_bytes-1); once its head names the
        # size, the rest of a bigger file is requested at once as up to `segments`
        # parallel Range streams (a file that fits stays one request).  0: open-ended
        # probe, one stream below `segment_threshold` (grab's behaviour)
        self.probe_bytes = max(0, probe_bytes)
        self.probe_mode = probe          # "get": ranged GET doubles as the probe; "head": grab-style HEAD first
        self.segments = max(1, segments)
        self.segment_threshold = segment_threshold
        self.chunk = chunk
        self.write_block = write_block
        self._session = session
        self.headers = headers or {"User-Agent": "tritondl/0.1"}
        self.max_retries = max_retries
        # a 429 / 503 whose Retry-After is at most this long is waited out inside the job
        # (it counts as a retry); a longer one fails the job, which the broker-side retry
        # path re-runs later with its own growing delay.  grab gave up on any status
        self.retry_after_max = 30.0
        # native data plane (csrc/relay): plain-http bodies go socket -> file in C++
        self.native = native
        self.read_timeout = read_timeout
        # splice(2) socket -> pipe -> file in the receive pump: one copy less, a win on ext4
        # (3.6 vs 5.9 ms per 10 MiB) but slower on the MI355X box's overlayfs with 4 concurrent
        # range streams (1 GiB fetch 154 vs 85 ms), so opt-in: TRITONDL_RELAY_SPLICE=1
        self.splice = os.environ.get("TRITONDL_RELAY_SPLICE", "0").lower() in ("1", "on", "true", "yes")
        # receive buffer of the native pump (socket -> buffer -> pwrite)
        self.recv_buf = int(os.environ.get("TRITONDL_RELAY_RECV_BUF", "") or (4 << 20))
        self._raw = rawhttp.Pool()
        # https trust: a private CA (PEM text / file), else the system store
        self.ca_pem, self.ca_file = ca_pem, ca_file or os.environ.get("TRITONDL_CA_FILE", "")
        self._ntls = None

    def _tls_ctx(self):
        if self._ntls is None:
            relay = rawhttp.relay_module()
            if self.ca_pem and relay is not None:
                self._ntls = relay.TlsContext.client(ca_pem=self.ca_pem)
            else:
                self._ntls = rawhttp.client_tls_context(self.ca_file)
        return self._ntls

    def register(self) -> ClientRegister:
        return ClientRegister(name="http", protocols=["http", "https"])

    async def _sess(self) -> aiohttp.ClientSession:
        if self._session is None or self._session.closed:
            ssl_ctx: object = True
            if self.ca_pem or self.ca_file:
                import ssl
                ssl_ctx = ssl.create_default_context(cafile=self.ca_file or None, cadata=self.ca_pem or None)
            self._session = aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=None, sock_connect=30, sock_read=120),
                connector=aiohttp.TCPConnector(limit=64, ssl=ssl_ctx, happy_eyeballs_delay=FALLBACK_DELAY,
                                             socket_factory=socket_factory), auto_decompress=False)
        return self._session

    async def close(self) -> None:
        for conns in list(self._h2conns.values()):
            for c in conns:
                await c.close()
        if self._h2closing:
            await asyncio.gather(*self._h2closing, return_exceptions=True)
        self._h2conns.clear()
        self._raw.close()
        if self._session is not None:
            await self._session.close()
            self._session = None

    # ------------------------------------------------------------ transport
    def _native_for(self, url: str):
        if not self.native or not url.startswith(("http://", "https://")):
            return None
        return rawhttp.relay_module()

    def _proxy(self, url: str) -> "_proxy.ProxyURL | None":
        """The egress proxy for ``url`` (grab's transport: ``ProxyFromEnvironment``)."""
        try:
            return (self.proxies or _proxy.from_environment()).proxy_for(url)
        except _proxy.ProxyConfigError as e:
            raise HTTPDownloadError(f"GET {url}: {e}") from e

    def _aio_proxy(self, url: str, headers: dict) -> dict:
        """aiohttp request kwargs (``headers`` included) routing ``url``
        through its proxy."""
        try:
            kw, extra = _proxy.aiohttp_kwargs(self._proxy(url), url.startswith("https:"))
        except ValueError as e:
            raise _FatalHTTPError(f"GET {url}: {e}") from e
        return {**kw, "headers": {**headers, **extra}}

    async def _aio_get(self, url: str, headers: dict):
        """aiohttp GET through the egress proxy; a proxy that refuses us
        (407/403 on CONNECT) fails the job instead of being retried."""
        s = await self._sess()
        try:
            return await s.get(url, allow_redirects=True, **self._aio_proxy(url, headers))
        except aiohttp.ClientHttpProxyError as e:
            if e.status in (401, 403, 407):
                raise _FatalHTTPError(f"GET {url}: proxy refused the tunnel: {e.status} {e.message}") from e
            raise

    async def _open(self, url: str, headers: dict):
        """GET ``url``: an :class:`_H2Response` when the origin speaks HTTP/2
        (``http2``), a :class:`_RawResponse` on the native path (plain
        http, identity body, no redirect), else an open aiohttp response."""
        if self.http2 and url.startswith("https://"):
            r = await self._h2_get(url, headers)
            if r is not None:
                return r
        if self._native_for(url) is not None:
            r = await self._raw_get(url, headers)
            if r is not None:
                return r
        r = await self._aio_get(url, headers)
        if r.status == 407:
            r.release()
            raise _FatalHTTPError(f"GET {url}: proxy authentication required (407)")
        return r

    def _h2_ssl(self):
        import ssl
        ctx = ssl.create_default_context(cafile=self.ca_file or None, cadata=self.ca_pem or None)
        return ctx

    def _h2_sweep(self) -> None:
        """Close HTTP/2 connections that died or sat without a stream for
        ``h2_idle_s``; forget expired HTTP/1.1-only verdicts."""
        now = time.monotonic()
        for key, conns in list(self._h2conns.items()):
            keep = []
            for c in conns:
                if not c.alive and not c.streams or c.idle_for(now) > self.h2_idle_s:
                    t = asyncio.ensure_future(c.close())
                    self._h2closing.add(t)
                    t.add_done_callback(self._h2closing.discard)
                else:
                    keep.append(c)
            if keep:
                self._h2conns[key] = keep
            else:
                del self._h2conns[key]
                lock = self._h2locks.get(key)
                if lock is not None and not lock.locked():
                    del self._h2locks[key]
        for key, until in list(self._h1_only.items()):
            if until <= now:
                del self._h1_only[key]

    def _h2_pick(self, key: tuple[str, int]) -> "_h2.H2Connection | None":
        """The least busy live connection to the origin, unless a new one
        should open (every one carries a stream and there are fewer than
        ``h2_conns``)."""
        conns = [c for c in self._h2conns.get(key, ()) if c.alive]
        if not conns:
            return None
        best = min(conns, key=lambda c: c.load)
        if best.load and len(conns) < self.h2_conns:
            return None
        best.pending += 1                            # the caller's request() settles it
        return best

    async def _h2_conn(self, host: str, port: int) -> "_h2.H2Connection | None":
        """A live HTTP/2 connection to the origin (see :meth:`_h2_pick`;
        opened on first use), or None if the origin speaks HTTP/1.1."""
        self._h2_sweep()
        key = (host, port)
        c = self._h2_pick(key)
        if c is not None:
            return c
        if time.monotonic() < self._h1_only.get(key, 0.0):
            return None
        lock = self._h2locks.setdefault(key, asyncio.Lock())
        async with lock:
            c = self._h2_pick(key)
            if c is not None:
                return c
            try:
                if self.h2_native and rawhttp.relay_module() is not None:
                    c = await _h2.H2Connection.open_native(host, port, self._tls_ctx(), timeout=30.0)
                else:
                    c = await _h2.H2Connection.open(host, port, self._h2_ssl(), timeout=30.0)
            except (OSError, RuntimeError, asyncio.TimeoutError) as e:
                raise aiohttp.ClientConnectionError(f"https://{host}:{port}: {e}") from e
            if c is None:
                self._h1_only[key] = time.monotonic() + 3600.0
                log.with_fields(origin=f"{host}:{port}").debug("origin does not speak HTTP/2; using HTTP/1.1")
                return None
            self._h2conns.setdefault(key, []).append(c)
            c.pending += 1
            return c

    async def _h2_get(self, url: str, headers: dict) -> "_H2Response | None":
        """GET over HTTP/2, following redirects like :meth:`_raw_get`; None
        when the origin (or a redirect target) does not speak it, or a proxy
        is in the way (the HTTP/1.1 paths handle those)."""
        for _hop in range(self.max_redirects + 1):
            u = URL(url)
            if u.scheme != "https" or self._proxy(url) is not None:
                return None
            host, port = u.raw_host or "", u.port or 443
            c = await self._h2_conn(host, port)
            if c is None:
                return None
            hh = {"Accept-Encoding": "identity",
                  **({} if "Authorization" in headers else rawhttp.basic_auth_header(u)), **headers}
            path = u.raw_path_qs or "/"
            fields = [(b":method", b"GET"), (b":scheme", b"https"), (b":authority", c.authority.encode()),
                      (b":path", path.encode())]
            fields += [(k.lower().encode(), str(v).encode()) for k, v in hh.items()
                       if k.lower() not in ("host", "connection", "keep-alive", "transfer-encoding", "upgrade")]
            st = None
            try:
                try:
                    st = await c.request(fields)
                finally:
                    c.pending -= 1
                await asyncio.wait_for(st.response(), self.read_timeout)
            except BaseException as e:
                if st is not None:
                    st.cancel()             # no head (timeout, error, the job cancelled): free the stream
                if isinstance(e, (_h2.H2Error, asyncio.TimeoutError)):
                    raise aiohttp.ClientConnectionError(f"GET {url} (HTTP/2): {e}") from e
                raise
            self.h2_streams += 1
            loc = st.headers.get("Location")
            if st.status in (301, 302, 303, 307, 308) and loc:
                st.cancel()
                try:
                    url = str(u.join(URL(loc)))
                except (ValueError, TypeError) as e:
                    raise HTTPDownloadError(f"GET {url}: bad redirect Location {loc!r}") from e
                continue
            if 300 <= st.status < 400:
                st.cancel()
                return None
            return _H2Response(st, url, self.read_timeout)
        raise HTTPDownloadError(f"GET {url}: stopped after {self.max_redirects} redirects")

    async def _raw_get(self, url: str, headers: dict) -> "_RawResponse | None":
        """Native GET.  Redirects (301/302/303/307/308, relative or absolute,
        http <-> https) are followed here, up to ``max_redirects`` like Go's
        http.Client under grab; the returned response's ``url`` is the final
        one (file naming uses it, as grab does)."""
        for _hop in range(self.max_redirects + 1):
            u = URL(url)
            secure = u.scheme == "https"
            dport = 443 if secure else 80
            host, port = u.raw_host or "", u.port or dport
            px = self._proxy(url)
            if not rawhttp.native_proxy_ok(px, secure):
                return None
            target = rawhttp.request_target(u, px, secure)
            hh = {"Host": host if port == dport else f"{host}:{port}", "Accept-Encoding": "identity",
                  **({} if "Authorization" in headers else rawhttp.basic_auth_header(u)), **headers,
                  **rawhttp.proxy_auth_header(px)}
            head = rawhttp.request_head("GET", target, hh)
            tls = self._tls_ctx() if secure else None
            if secure and tls is None:
                return None
            h = conn = None
            for _ in range(2):                # a stale pooled keep-alive connection gets one fresh retry
                try:
                    conn, reused = await self._raw.connect(
                        host, port, timeout=30.0, tls=tls, proxy=px,
                        proxy_tls=self._tls_ctx() if px is not None and px.scheme == "https" else None)
                except rawhttp.ProxyRefused as e:
                    raise _FatalHTTPError(f"GET {url}: {e}") from e
                except (OSError, rawhttp.RawHTTPError) as e:
                    raise aiohttp.ClientConnectionError(f"GET {url}: {e}") from e
                try:
                    await conn.sendall(head, self.read_timeout)
                    rawhttp.trace("get_sent")
                    h = await rawhttp.read_head(conn, self.read_timeout)
                    rawhttp.trace("get_head")
                    break
                except (OSError, rawhttp.RawHTTPError) as e:
                    conn.close()
                    if reused:
                        continue
                    raise aiohttp.ClientConnectionError(str(e)) from e
                except BaseException:
                    conn.close()
                    raise
            if h is None:
                raise aiohttp.ClientConnectionError(f"GET {url}: connection reset")
            if h.status == 407 and rawhttp.absolute_form(px):
                conn.close()
                raise _FatalHTTPError(f"GET {url}: proxy {px.redacted()} requires authentication: "
                                      f"407 {h.reason}")
            loc = h.headers.get("Location")
            if h.status in (301, 302, 303, 307, 308) and loc:
                conn.close()                  # small redirect body: not worth draining for keep-alive
                try:
                    url = str(u.join(URL(loc)))
                except (ValueError, TypeError) as e:
                    raise HTTPDownloadError(f"GET {url}: bad redirect Location {loc!r}") from e
                if not url.startswith(("http://", "https://")):
                    return None
                continue
            if 300 <= h.status < 400:
                conn.close()                  # odd 3xx (300, 304, ...): aiohttp handles these
                return None
            # chunked bodies are decoded by the native pump; a content-coded body is
            # stored as sent, like the aiohttp path (auto_decompress=False) stores it
            return _RawResponse(self._raw, host, port, conn, h, url)
        raise HTTPDownloadError(f"GET {url}: stopped after {self.max_redirects} redirects")

    # ------------------------------------------------------------ probe
    async def _probe(self, url: str) -> _Probe:
        s = await self._sess()
        try:
            async with s.head(url, allow_redirects=True, **self._aio_proxy(url, self.headers)) as r:
                if r.status < 400:
                    return self._probe_from(r, url)
        except aiohttp.ClientError:
            pass
        # HEAD unsupported: probe with a 1-byte ranged GET
        async with await self._aio_get(url, {**self.headers, "Range": "bytes=0-0"}) as r:
            if r.status == 407:
                raise _FatalHTTPError(f"GET {url}: proxy authentication required (407)")
            if r.status >= 400:
                raise HTTPDownloadError(f"GET {url}: HTTP {r.status}")
            p = self._probe_from(r, url)
            if r.status == 206:
                cr = r.headers.get("Content-Range", "")
                m = re.match(r"bytes \d+-\d+/(\d+)", cr)
                p.size = int(m.group(1)) if m else None
                p.ranges = True
            return p

    async def _probe_get(self, url: str) -> tuple[_Probe, aiohttp.ClientResponse | None]:
        """Probe with ``GET Range: bytes=0-`` and keep the response open: its
        body becomes the first segment's stream, saving the HEAD round trip
        (one RTT per job — the whole cost of a small job on a distant origin)."""
        s = await self._sess()
        attempt = 0
        while True:
            try:
                rng = f"bytes=0-{self.probe_bytes - 1}" if self.probe_bytes else "bytes=0-"
                r = await self._open(url, {**self.headers, "Range": rng})
                if r.status == 416:                      # empty resource: no satisfiable range
                    r.release()
                    r = await self._open(url, dict(self.headers))
                wait = retry_after(r)
                if r.status < 500 and wait is None:
                    break
                r.release()
                err: Exception = HTTPDownloadError(f"GET {url}: HTTP {r.status}")
            except (aiohttp.ClientError, asyncio.TimeoutError) as e:
                err, wait = e, None
            attempt += 1                                 # 5xx / 429 / transport error: transient
            if attempt > self.max_retries:
                raise HTTPDownloadError(f"probe of {url} failed: {err}") from err
            if wait is not None and wait > self.retry_after_max:
                raise HTTPDownloadError(f"GET {url}: HTTP {getattr(r, 'status', '?')}, retry after {wait:.0f}s")
            d = min(0.2 * 2 ** attempt, 5.0) if wait is None else wait
            log.with_fields(error=str(err), attempt=attempt, delay_s=round(d, 2)).warn("download probe failed; retrying")
            await asyncio.sleep(d)
        if r.status >= 400:
            r.release()
            raise HTTPDownloadError(f"GET {url}: HTTP {r.status}")
        try:
            p = self._probe_from(r, url)
        except BaseException:
            r.release()
            raise
        if r.status == 206:
            m = re.match(r"bytes (\d+)-(\d+)/(\d+)", r.headers.get("Content-Range", ""))
            if not m or m.group(1) != "0":
                r.release()
                raise HTTPDownloadError(f"GET {url}: bad Content-Range {r.headers.get('Content-Range')!r}")
            p.size, p.ranges, p.first_end = int(m.group(3)), True, int(m.group(2)) + 1
        # aiohttp reports the URL without its userinfo: that is not a redirect, and
        # the Range requests must keep the credentials (Go's later requests do)
        if str(r.url) != url and str(r.url) != str(URL(url).with_user(None)):
            p.final_url = str(r.url)
        return p, r

    def _probe_from(self, r: aiohttp.ClientResponse, url: str) -> _Probe:
        size = r.headers.get("Content-Length")
        if "chunked" in r.headers.get("Transfer-Encoding", "").lower():
            size = None                 # RFC 9112 §6.3: chunked framing overrides Content-Length
        name = filename_from_disposition(r.headers.get("Content-Disposition")) or \
            filename_from_url(str(r.url)) or filename_from_url(url)
        if not name:
            raise HTTPDownloadError("no filename could be determined")
        if size is not None:
            size = size.split(",")[0].strip()            # "42, 42": a repeated, identical length
            if not (size.isascii() and size.isdigit()):
                raise HTTPDownloadError(f"GET {url}: bad Content-Length {r.headers.get('Content-Length')!r}")
        return _Probe(int(size) if size is not None and r.status == 200 else None,
                      r.headers.get("Accept-Ranges", "").lower() == "bytes", r.headers.get("ETag", ""),
                      r.headers.get("Last-Modified", ""), name, r.status)

    # ------------------------------------------------------------ download
    async def download(self, base_dir: str, progress: ProgressSink, url: str) -> None:
        h = await self.start(base_dir, progress, url)
        await h.wait()

    async def start(self, base_dir: str, progress: ProgressSink, url: str) -> "DownloadHandle":
        """Probe and start the transfer; returns a handle exposing the
        destination, the size and a contiguous-bytes watermark so a consumer
        (the streaming uploader) can read the file while it is written."""
        first: aiohttp.ClientResponse | None = None
        if self.probe_mode == "head":
            probe = await self._probe(url)
        else:
            probe, first = await self._probe_get(url)
        dst = os.path.join(base_dir, probe.filename)
        part, meta_path = dst + ".part", dst + ".part.meta"
        if probe.size is not None and os.path.exists(dst) and os.path.getsize(dst) == probe.size:
            if first is not None:
                first.close()
            log.with_field("file", dst).info("file already downloaded; skipping")
            progress(url, 100)
            return DownloadHandle.finished(dst, probe.size)
        validator = probe.etag or probe.last_modified
        segs = self._plan(probe)
        meta = self._load_meta(meta_path)
        resumable = (isinstance(meta, dict) and os.path.exists(part) and probe.ranges and validator and
                     meta.get("url") == url and meta.get("validator") == validator and
                     meta.get("size") == probe.size and _segments_ok(meta.get("segments"), probe.size))
        if resumable:
            segs = [list(x) for x in meta["segments"]]
            log.with_fields(file=dst, done=sum(s[2] for s in segs)).info("resuming download")
            if first is not None:                # resume uses ranged requests with If-Range
                first.close()
                first = None
        if probe.size:
            have = sum(sg[2] for sg in segs) if resumable else 0
            try:
                try:
                    check_space(base_dir, probe.size - have, self.disk_reserve)
                except DiskSpaceError:
                    pool = spares.pool_for(base_dir)
                    if pool is None or not pool.release():
                        raise
                    check_space(base_dir, probe.size - have, self.disk_reserve)   # spares deleted: again
            except DiskSpaceError as e:
                if first is not None:
                    first.close()
                raise HTTPDownloadError(str(e)) from e
        if not resumable:
            # a spare (a finished job's file, --cleanup only) is overwritten in place:
            # its page cache is reused instead of freed and allocated again (utils/spares.py)
            pool = spares.pool_for(base_dir) if probe.size else None
            if pool is not None and pool.take(part):
                fd = os.open(part, os.O_WRONLY)
            else:
                fd = os.open(part, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            try:
                if probe.size:
                    os.ftruncate(fd, probe.size)
            finally:
                os.close(fd)
        h = DownloadHandle(dst, part, probe.size, segs)
        h.task = asyncio.ensure_future(self._run(h, probe, url, validator, meta_path, progress, first))
        return h

    async def _run(self, h: "DownloadHandle", probe: _Probe, url: str, validator: str, meta_path: str,
                   progress: ProgressSink, first: aiohttp.ClientResponse | None = None) -> None:
        segs, done = h.segs, h.done
        state = {"url": url, "validator": validator, "size": probe.size, "segments": segs}
        t0 = time.monotonic()

        def sync_save() -> None:
            for k, sg in enumerate(segs):
                sg[2] = h.seg_done(k)
            self._save_meta(meta_path, state)

        async def reporter() -> None:
            while True:
                await asyncio.sleep(self.progress_interval)
                tot = probe.size or 0
                pct = (sum(h.seg_done(k) for k in range(len(segs))) / tot * 100) if tot else 0.0
                progress(url, min(pct, 99.99))
                sync_save()

        fd = os.open(h.part, os.O_WRONLY)
        rep = asyncio.ensure_future(reporter())
        src = probe.final_url or url          # follow-up ranges skip the redirect hop(s)
        # a single stream runs inline, so its receive pump starts in this task's
        # first step, ahead of a streamed upload's first step (SigV4 setup,
        # connection): the upload then follows a download already running
        # instead of delaying it, 427.7 vs 395.1 jobs/s (profiles/r05_gil_ab/,
        # r05_inline_ab/).  Round 2 measured the opposite order faster, before
        # the signed sender followed the download's frontier.
        inline = None
        if len(segs) == 1:
            tasks = []
            inline = self._fetch_segment(src, fd, 0, segs, done, validator, probe, h, first)
        elif len(segs) <= self.segments:
            tasks = [asyncio.ensure_future(self._fetch_segment(src, fd, i, segs, done, validator, probe, h,
                                                               first if i == 0 else None))
                     for i in range(len(segs))]
        else:
            # stripes: `segments` stream workers take the next stripe in file order
            order = iter(range(len(segs)))

            async def worker() -> None:
                for i in order:
                    await self._fetch_segment(src, fd, i, segs, done, validator, probe, h,
                                              first if i == 0 else None)
            tasks = [asyncio.ensure_future(worker()) for _ in range(self.segments)]
        try:
            if inline is not None:
                await inline
            else:
                await asyncio.gather(*tasks)
        except BaseException as e:
            # stop every sibling and WAIT for it: their native pumps write through
            # `fd` and read their own sockets, which must stay open until they return
            h._fail(e)                       # the error a following upload reports
            if h.flow is not None:
                h.flow.cancel()
            for t in tasks:
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
            if first is not None:
                first.close()
            sync_save()
            raise
        finally:
            rep.cancel()
            os.close(fd)
        total = sum(done)
        if probe.size is not None and total != probe.size:
            err = HTTPDownloadError(f"short download: {total} of {probe.size} bytes")
            h._fail(err)
            raise err
        if probe.size is None:
            os.truncate(h.part, total)
        os.replace(h.part, h.dst)
        _set_remote_time(h.dst, probe.last_modified)
        try:
            os.remove(meta_path)
        except FileNotFoundError:
            pass
        h._finish(total)
        dt = time.monotonic() - t0
        log.with_fields(file=h.dst, bytes=total, mbps=round(total / max(dt, 1e-9) / 1e6, 1)).info("download finished")
        progress(url, 100)

    def _plan(self, p: _Probe) -> list[list[int]]:
        """[[start, end_exclusive_or_-1, done], ...]"""
        if p.size is None:
            return [[0, -1, 0]]
        if self.probe_bytes and p.ranges and p.first_end is not None:
            # bounded GET probe: its body is segment 0; the rest goes to up to
            # `segments - 1` further Range streams, none shorter than the probe's body
            if p.first_end >= p.size:
                return [[0, p.size, 0]]
            rest = p.size - p.first_end
            if self.stripe_bytes:
                st = self.stripe_bytes
                return [[0, p.first_end, 0]] + [[a, min(p.size, a + st), 0] for a in range(p.first_end, p.size, st)]
            # the probe is one of the `segments` streams: at most segments-1 more
            k = max(1, min(max(1, self.segments - 1), -(-rest // p.first_end)))
            step = -(-rest // k)
            return [[0, p.first_end, 0]] + [[p.first_end + i * step, min(p.size, p.first_end + (i + 1) * step), 0]
                                            for i in range(k) if p.first_end + i * step < p.size]
        n = self.segments if (p.ranges and p.size >= self.segment_threshold) else 1
        if n > 1 and self.stripe_bytes:
            st = self.stripe_bytes
            return [[a, min(p.size, a + st), 0] for a in range(0, p.size, st)]
        step = -(-p.size // n)
        return [[i * step, min(p.size, (i + 1) * step), 0] for i in range(n) if i * step < p.size] or [[0, 0, 0]]

    @staticmethod
    def _load_meta(path: str) -> dict | None:
        try:
            with open(path) as f:
                return json.load(f)
        except (OSError, ValueError):
            return None

    @staticmethod
    def _save_meta(path: str, state: dict) -> None:
        tmp = path + ".tmp"
        try:
            with open(tmp, "w") as f:
                json.dump(state, f)
            os.replace(tmp, path)
        except OSError:
            pass

    async def _fetch_segment(self, url: str, fd: int, i: int, segs: list[list[int]], done: list[int],
                             validator: str, probe: _Probe, h: "DownloadHandle | None" = None,
                             first: aiohttp.ClientResponse | None = None) -> None:
        start, end, _ = segs[i]
        attempt = 0
        while True:
            pos = start + done[i]
            if end >= 0 and pos >= end:
                if first is not None:
                    first.close()
                return
            try:
                if first is not None and pos == 0:
                    # the probe's open response already streams from byte 0
                    r, first = first, None
                    try:
                        await self._consume(r, fd, i, segs, done, h, 0, end)
                    except BaseException:
                        r.close()
                        raise
                    if len(segs) == 1 or end == probe.first_end:
                        r.release()          # body read to its end: keep-alive connection back to the pool
                    else:
                        r.close()            # stopped mid-body at the segment boundary: drop it
                    return
                hdrs = dict(self.headers)
                if pos > 0 or end >= 0 and len(segs) > 1:
                    hdrs["Range"] = f"bytes={pos}-" + (f"{end - 1}" if end >= 0 else "")
                    if validator:
                        hdrs["If-Range"] = validator
                r = await self._open(url, hdrs)
                try:
                    wait = retry_after(r)
                    if wait is not None:
                        raise _RetryLater(f"GET {url}: HTTP {r.status}, retry after {wait:.1f}s", wait)
                    if r.status >= 400:
                        raise HTTPDownloadError(f"GET {url}: HTTP {r.status}")
                    if "Range" in hdrs and r.status != 206:
                        if len(segs) > 1 or pos > 0:
                            if len(segs) == 1:  # origin ignored Range: restart from zero
                                done[i] = 0
                                pos = 0
                            else:
                                raise _FatalHTTPError("origin ignored Range request")
                    await self._consume(r, fd, i, segs, done, h, pos, end)
                finally:
                    r.release()
                return
            except (aiohttp.ClientError, asyncio.TimeoutError, HTTPDownloadError, ConnectionError) as e:
                attempt += 1
                if h is not None and h.flow is not None and h.flow.cancelled:
                    raise _FatalHTTPError(f"segment {i} of {url}: download cancelled") from e
                later = e.after if isinstance(e, _RetryLater) else None
                if attempt > self.max_retries or isinstance(e, _FatalHTTPError) or \
                        (later is not None and later > self.retry_after_max) or \
                        (later is None and isinstance(e, HTTPDownloadError) and "HTTP 4" in str(e)):
                    raise HTTPDownloadError(f"segment {i} of {url} failed: {e}") from e
                d = min(0.2 * 2 ** attempt, 5.0) if later is None else later
                log.with_fields(error=str(e), attempt=attempt, segment=i).warn("download stream failed; retrying")
                await asyncio.sleep(d)

    async def _consume(self, r, fd: int, i: int, segs: list[list[int]], done: list[int],
                       h: "DownloadHandle | None", pos: int, end: int) -> None:
        """Stream one response body into the file at ``pos`` (up to ``end``)."""
        if isinstance(r, _RawResponse):
            return await self._consume_native(r, fd, i, segs, done, h, pos, end)
        loop = asyncio.get_running_loop()
        start = segs[i][0]
        limit = (end - pos) if end >= 0 else -1
        if isinstance(r, _H2Response) and r.st.conn.native:
            return await self._consume_h2_native(r, i, segs, done, h, fd, pos, end, limit)
        if limit >= 0 and isinstance(r, _H2Response):
            r.st.want(limit)
        bufs: list[bytes] = []
        nbuf = 0
        wpos = pos
        async for chunk in r.content.iter_chunked(self.chunk):
            if limit >= 0:
                room = limit - (wpos - pos) - nbuf
                if len(chunk) > room:
                    chunk = chunk[:room]       # probe stream runs past this segment
            if chunk:
                bufs.append(chunk)
                nbuf += len(chunk)
            if nbuf >= self.write_block or (limit >= 0 and (wpos - pos) + nbuf >= limit):
                await rawhttp.run_settled(loop, _pwritev_all, fd, bufs, wpos)
                wpos += nbuf
                done[i] += nbuf
                bufs, nbuf = [], 0
                if h is not None:
                    h._advance(i, done[i])
                if limit >= 0 and wpos - pos >= limit and not r.content.at_eof():
                    if segs[i][1] < 0 or len(segs) > 1:
                        break               # more body follows (next segment's bytes): stop here
        if bufs:
            await rawhttp.run_settled(loop, _pwritev_all, fd, bufs, wpos)
            wpos += nbuf
            done[i] += nbuf
            if h is not None:
                h._advance(i, done[i])
        if end >= 0 and start + done[i] < end:
            raise HTTPDownloadError("connection closed early")

    async def _consume_h2_native(self, r: "_H2Response", i: int, segs: list[list[int]], done: list[int],
                                 h: "DownloadHandle | None", fd: int, pos: int, end: int, limit: int) -> None:
        """An HTTP/2 stream on a native connection: the session pump writes
        the body into the file and onto the handle's flow (csrc/relay/h2.h)."""
        flow = h.flow if h is not None else None
        rawhttp.trace("get_pump_start")
        try:
            got, eof = await r.st.sink(fd, pos, limit, flow, i, done[i], self.read_timeout)
            rawhttp.trace("get_pump_end")
        except _h2.H2Error as e:
            done[i] += e.written
            if h is not None:
                h._advance(i, done[i])
            raise aiohttp.ClientConnectionError(str(e)) from e
        done[i] += got
        if h is not None:
            h._advance(i, done[i])
        if not eof:
            r.st.cancel()                           # the probe stream runs on into the next segment
        if end >= 0 and segs[i][0] + done[i] < end:
            raise HTTPDownloadError("connection closed early")

    async def _consume_native(self, r: _RawResponse, fd: int, i: int, segs: list[list[int]], done: list[int],
                              h: "DownloadHandle | None", pos: int, end: int) -> None:
        """The body goes socket -> file inside ``_relay.recv_body`` (GIL
        released), which publishes progress on the handle's native flow."""
        relay = rawhttp.relay_module()
        limit = (end - pos) if end >= 0 else -1
        cl = r.head.content_length
        if limit >= 0:
            n = min(limit, cl) if cl is not None else limit
        else:
            n = cl if cl is not None else -1
        prefix, r.leftover = r.leftover, b""
        flow = h.flow if h is not None else None
        chunked = r.head.chunked
        rawhttp.trace("get_pump_start")
        res = await rawhttp.run_pump(
            r.sock, relay.recv_body, fd, pos, n, prefix, flow, i, done[i], self.read_timeout, self.recv_buf,
            self.splice, chunked)
        rawhttp.trace("get_pump_end")
        got, eof, err = res[:3]
        done[i] += got
        if h is not None:
            h._advance(i, done[i])
        if err:
            r.close()
            if err == "cancelled" or (flow is not None and flow.cancelled):
                raise _FatalHTTPError(f"segment {i}: cancelled")
            raise HTTPDownloadError(err)
        if chunked:
            r.complete = bool(res[3])             # last chunk read, nothing after it: reusable
        else:
            r.complete = (n < 0 and eof) or (cl is not None and n == cl and len(prefix) <= cl)
            if n < 0:
                r.head.keep_alive = False         # close-delimited body
        if end >= 0 and segs[i][0] + done[i] < end:
            raise HTTPDownloadError("connection closed early")


class DownloadHandle:
    """A running (or finished) HTTP transfer.  ``watermark()`` is the length
    of the contiguous prefix already on disk; ``wait_bytes(n)`` blocks until
    n bytes are readable (or the transfer fails)."""

    def __init__(self, dst: str, part: str, size: int | None, segs: list[list[int]]) -> None:
        self.dst = dst
        self.part = part
        self.size = size
        self.segs = segs
        self.done = [s[2] for s in segs]
        self.task: asyncio.Task | None = None
        self._event = asyncio.Event()
        self._error: BaseException | None = None
        self._complete = False
        self._read_fd: int | None = None
        relay = rawhttp.relay_module()
        # native progress shared with the relay pumps (None without the extension)
        self.flow = relay.Flow([(st, en, d) for st, en, d in segs]) if relay is not None else None

    @classmethod
    def finished(cls, dst: str, size: int) -> "DownloadHandle":
        h = cls(dst, dst, size, [[0, size, size]])
        h._complete = True
        return h

    @property
    def filename(self) -> str:
        return os.path.basename(self.dst)

    def watermark(self) -> int:
        if self._complete:
            return self.size or 0
        if self.flow is not None:
            return self.flow.watermark()
        w = 0
        for (start, end, _d), done in zip(self.segs, self.done):
            w = start + done
            if end < 0 or start + done < end:
                break
        return w

    def _advance(self, i: int, done: int) -> None:
        if self.flow is not None:
            self.flow.advance(i, done)
        self._event.set()

    def seg_done(self, i: int) -> int:
        """Bytes of segment i on disk (the native pump advances the flow
        while it runs; ``done`` catches up when it returns)."""
        d = self.done[i]
        return max(d, self.flow.done(i)) if self.flow is not None else d

    def _fail(self, e: BaseException) -> None:
        self._error = e
        if self.flow is not None:
            self.flow.fail(str(e) or type(e).__name__)
        self._event.set()

    def _finish(self, total: int) -> None:
        self.size = total
        self._complete = True
        if self.flow is not None:
            self.flow.finish(total)
        self._event.set()

    async def wait_bytes(self, n: int) -> None:
        if self.flow is not None and not self._complete:
            loop = asyncio.get_running_loop()
            while True:
                if self._error is not None:
                    raise HTTPDownloadError(f"source transfer failed: {self._error}")
                r = await loop.run_in_executor(None, self.flow.wait_covered, 0, n, 0.5)
                if r == 0:
                    return
                if r == 1:
                    raise HTTPDownloadError(f"source transfer failed: {self._error or self.flow.error}")
                if r == 3:
                    raise HTTPDownloadError("source shorter than expected")
        while self.watermark() < n:
            if self._error is not None:
                raise HTTPDownloadError(f"source transfer failed: {self._error}")
            if self._complete:
                raise HTTPDownloadError("source shorter than expected")
            self._event.clear()
            await self._event.wait()

    def open_reader(self) -> int:
        """An fd on the file being written (stays valid across the final rename)."""
        if not self._complete:
            try:
                return os.open(self.part, os.O_RDONLY)
            except FileNotFoundError:  # renamed to dst in between
                pass
        return os.open(self.dst, os.O_RDONLY)

    async def wait(self) -> None:
        if self.task is not None:
            await self.task

    def cancel(self) -> None:
        if self.flow is not None:
            self.flow.cancel()             # stops native pumps blocked on this download
        if self.task is not None and not self.task.done():
            self.task.cancel()


def _set_remote_time(path: str, last_modified: str) -> None:
    """grab's ``setLastModified`` (``IgnoreRemoteTime`` is false by default):
    a parseable ``Last-Modified`` becomes the file's atime and mtime."""
    if not last_modified:
        return
    from email.utils import parsedate_to_datetime
    try:
        t = parsedate_to_datetime(last_modified).timestamp()
        os.utime(path, (t, t))
    except (TypeError, ValueError, OverflowError, OSError):
        pass


def _pwritev_all(fd: int, bufs: list[bytes], pos: int) -> None:
    """Vectored write of the received chunks — no concatenation copy."""
    total = sum(len(b) for b in bufs)
    n = os.pwritev(fd, bufs, pos)
    if n < total:  # short write: finish the remainder the slow way
        _pwrite_all(fd, b"".join(bufs)[n:], pos + n)


def _pwrite_all(fd: int, data: bytes, pos: int) -> None:
    mv = memoryview(data)
    while mv:
        n = os.pwrite(fd, mv, pos)
        mv = mv[n:]
        pos += n
