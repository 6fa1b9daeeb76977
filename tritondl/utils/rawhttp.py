"""HTTP/1.1 plumbing for the native data plane (``csrc/relay/``).

The control plane stays in asyncio: connect (and, for ``https``, drive the
TLS handshake), write a request head, parse a response head, read small
bodies (S3 replies).  Large bodies never pass through Python — the
connection's native stream (``_relay.Sock`` or ``_relay.TlsConn``) is handed
to ``_relay.recv_body`` / ``_relay.send_body``, which run in an executor
thread with the GIL released.  While a pump owns a connection, asyncio does
not touch it; :func:`run_pump` makes sure a cancelled caller stops the pump
and waits for it before the socket or file can be closed.

TLS is OpenSSL inside the relay module (non-blocking steps driven from the
event loop for handshakes and heads; the pumps encrypt/decrypt off-loop), so
``https`` origins and S3 endpoints keep the native path.  Scope (everything
else falls back to aiohttp in the callers): identity transfer coding for
downloads, no redirects.  Idle keep-alive connections are pooled per
(host, port, tls).
"""

from __future__ import annotations

import asyncio
import base64
import os
import socket
import time
import weakref
from dataclasses import dataclass, field

from multidict import CIMultiDict

from . import dial
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


class ProxyError(RawHTTPError):
    """The egress proxy could not be reached or could not open the tunnel
    (transient: 502/503/504 from CONNECT, a connect failure)."""


class ProxyRefused(ProxyError):
    """The proxy refused this client (407 / 403 on CONNECT, SOCKS auth or rule
    refusal): retrying cannot help, so callers fail the job at once."""

    def __init__(self, msg: str, status: int = 0) -> None:
        super().__init__(msg)
        self.status = status


def absolute_form(proxy) -> bool:
    """Requests go to an http(s) proxy in absolute form (``GET http://h/p``)
    for plain-http targets; https targets and socks5 use a tunnel."""
    return proxy is not None and proxy.scheme in ("http", "https")


def request_target(url, proxy, secure: bool) -> str:
    """Request-line target of ``url`` (a yarl URL): origin form, or absolute
    form when it goes through an http(s) proxy without a tunnel."""
    if not secure and absolute_form(proxy):
        return str(url.with_fragment(None).with_user(None))     # userinfo never goes on the wire
    return url.raw_path_qs or "/"


def basic_auth_header(url) -> dict:
    """Go's http.Client sends a URL's userinfo as ``Authorization: Basic``
    (``net/http/client.go`` ``send``) on that request only: a redirect to a
    URL without userinfo goes without it.  ``url`` is a yarl URL (user and
    password percent-decoded, as Go's ``Username()`` / ``Password()``)."""
    if url.user is None:
        return {}
    raw = f"{url.user}:{url.password or ''}".encode()
    return {"Authorization": "Basic " + base64.b64encode(raw).decode()}


def native_proxy_ok(proxy, secure: bool) -> bool:
    """False for TLS inside TLS (an https target through an https proxy),
    which the native streams do not do; callers use aiohttp then."""
    return not (secure and proxy is not None and proxy.scheme == "https")


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
        """None when absent, malformed, or overridden by chunked
        Transfer-Encoding (RFC 9112 §6.3: Content-Length is then ignored)."""
        if self.chunked:
            return None
        v = self.headers.get("Content-Length")
        try:
            return int(v.split(",")[0]) if v is not None else None
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
    if sep and p.isascii() and p.isdigit() and ":" not in h:
        return h, int(p)
    return hostport, default_port


class RawConn:
    """A connected, non-blocking stream: a plain socket, or a TLS session
    (``_relay.TlsConn``) over one.  ``native`` is what the relay pumps take.
    Owns the socket; :meth:`close` closes it."""

    pool_key: tuple | None = None

    def __init__(self, sock: socket.socket, tls=None) -> None:
        self.sock = sock
        self.tls = tls
        relay = relay_module()
        self.native = tls if tls is not None else (relay.Sock(sock.fileno()) if relay is not None else None)
        self._loop = asyncio.get_running_loop()

    @property
    def secure(self) -> bool:
        return self.tls is not None

    def fileno(self) -> int:
        return self.sock.fileno()

    async def _wait(self, events: int, timeout: float | None = None) -> None:
        """Wait until the socket is readable (POLLIN=1) / writable (POLLOUT=4);
        asyncio.TimeoutError after ``timeout`` seconds (a timer handle, not a
        wait_for task: this sits on every request's critical path)."""
        fut = self._loop.create_future()
        fd = self.sock.fileno()

        def ready() -> None:
            if not fut.done():
                fut.set_result(None)

        def expire() -> None:
            if not fut.done():
                fut.set_exception(asyncio.TimeoutError())

        rd, wr = bool(events & 1), bool(events & 4)
        if rd:
            self._loop.add_reader(fd, ready)
        if wr:
            self._loop.add_writer(fd, ready)
        timer = self._loop.call_later(timeout, expire) if timeout is not None else None
        try:
            await fut
        finally:
            if timer is not None:
                timer.cancel()
            if rd:
                self._loop.remove_reader(fd)
            if wr:
                self._loop.remove_writer(fd)

    async def handshake(self, timeout: float) -> None:
        async def go() -> None:
            while True:
                try:
                    w = self.tls.handshake_step()
                except RuntimeError as e:
                    raise RawHTTPError(str(e)) from e
                if w == 0:
                    return
                await self._wait(w)
        try:
            await asyncio.wait_for(go(), timeout)
        except asyncio.TimeoutError as e:
            raise RawHTTPError("tls handshake timed out") from e

    async def recv(self, n: int, timeout: float | None = None) -> bytes:
        """Up to n bytes; b"" at end of stream.  Tries the (non-blocking)
        socket first and waits only if nothing is there yet; ``timeout``
        bounds each wait (asyncio.TimeoutError)."""
        if self.tls is None:
            while True:
                try:
                    return self.sock.recv(n)
                except (BlockingIOError, InterruptedError):
                    await self._wait(1, timeout)
        while True:
            try:
                r = self.tls.read_nb(n)
            except RuntimeError as e:
                raise RawHTTPError(str(e)) from e
            if isinstance(r, bytes):
                return r
            await self._wait(r, timeout)

    async def sendall(self, data: bytes, timeout: float | None = None) -> None:
        """Send everything; a request head normally leaves in one ``send``
        with no event-loop round trip."""
        mv = memoryview(data)
        if self.tls is None:
            while mv:
                try:
                    k = self.sock.send(mv)
                except (BlockingIOError, InterruptedError):
                    k = 0
                if k:
                    mv = mv[k:]
                else:
                    await self._wait(4, timeout)
            return
        while mv:
            try:
                n, want = self.tls.write_nb(bytes(mv))
            except RuntimeError as e:
                raise RawHTTPError(str(e)) from e
            if n:
                mv = mv[n:]
            else:
                await self._wait(want, timeout)
        while True:                      # ciphertext the TLS layer still holds
            try:
                want = self.tls.flush_nb()
            except RuntimeError as e:
                raise RawHTTPError(str(e)) from e
            if not want:
                return
            await self._wait(want, timeout)

    def alive(self) -> bool:
        """Idle pooled connection still usable (peer has not closed it)."""
        if self.tls is not None:
            try:
                return self.tls.alive()
            except RuntimeError:
                return False
        try:
            self.sock.recv(1, socket.MSG_PEEK | socket.MSG_DONTWAIT)
            return False         # EOF, or stray bytes: not reusable either way
        except BlockingIOError:
            return True          # nothing pending, still open
        except OSError:
            return False

    def abort(self) -> None:
        """Stop a pump running on this connection without closing the fd."""
        if self.native is not None:
            self.native.abort()
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass

    def close(self) -> None:
        if self.sock.fileno() < 0:
            return
        if self.tls is not None:
            try:
                self.tls.shutdown_notify()
            except RuntimeError:
                pass
        self.sock.close()


@dataclass
class Pool:
    """Idle keep-alive connections by (host, port, tls) — or, through an
    egress proxy, by (proxy) for absolute-form requests and by (proxy,
    host, port, tls) for tunnels."""
    max_idle: int = 16
    idle: dict = field(default_factory=dict)
    # Go's http.Transport closes a connection idle for 90 s (IdleConnTimeout) and keeps at most
    # 100 idle in all: a worker that meets thousands of origins must not keep a socket for each
    idle_s: float = 90.0
    max_idle_total: int = 100
    _next_sweep: float = 0.0

    async def connect(self, host: str, port: int, timeout: float = 30.0, tls=None,
                      server_hostname: str | None = None, proxy=None, proxy_tls=None) -> tuple[RawConn, bool]:
        """(connection, reused).  ``tls``: a ``_relay.TlsContext`` (client) for
        https.  A pooled connection the peer has closed is dropped.

        ``proxy`` (a :class:`~tritondl.utils.proxy.ProxyURL`): for a plain-http
        target through an http(s) proxy the connection goes to the proxy (the
        caller sends absolute-form requests with :func:`proxy_auth_header`);
        for an https target the proxy is asked to ``CONNECT host:port`` and
        TLS runs inside the tunnel; ``socks5`` opens a SOCKS tunnel either way.
        ``proxy_tls``: the client context for an ``https://`` proxy (Go uses
        the transport's TLS config, i.e. the same trust as for targets;
        default: the shared system-store context).
        """
        self.sweep()
        tid = id(tls) if tls is not None else 0
        if proxy is None:
            key: tuple = (host, port, tid)
        elif tls is None and absolute_form(proxy):
            key = ("proxy",) + proxy.key
        else:
            key = ("tunnel",) + proxy.key + (host, port, tid)
        lst = self.idle.get(key)
        while lst:
            c = lst.pop()
            if c.alive():
                return c, True
            c.close()
        if proxy is None:
            s = await _dial(host, port, timeout)
        else:
            try:
                s = await _dial(proxy.host, proxy.port, timeout)
            except RawHTTPError as e:
                raise ProxyError(f"proxyconnect tcp: {proxy.redacted()}: {e}") from e
        try:
            if proxy is not None and proxy.scheme == "https":
                if tls is not None:
                    raise ProxyError("TLS inside an https proxy tunnel is not supported natively")
                c = RawConn(s, relay_module().TlsConn(proxy_tls or client_tls_context(), s.fileno(), proxy.host,
                                                     f"{proxy.host}:{proxy.port}"))
                await c.handshake(timeout)
                c.pool_key = key
                return c, False
            if proxy is not None and proxy.scheme == "socks5":
                await _socks5_connect(RawConn(s), proxy, host, port, timeout)
            elif proxy is not None and tls is not None:
                await _http_connect(RawConn(s), proxy, host, port, timeout)
            if tls is None:
                c = RawConn(s)
                c.pool_key = key
                return c, False
            t = relay_module().TlsConn(tls, s.fileno(), server_hostname or host, f"{host}:{port}")
            c = RawConn(s, t)
            await c.handshake(timeout)
        except asyncio.TimeoutError as e:
            s.close()
            raise (ProxyError if proxy is not None else RawHTTPError)(
                f"connect {_hostport(host, port)}: timed out") from e
        except BaseException:
            s.close()
            raise
        c.pool_key = key
        return c, False

    def release(self, host: str, port: int, c: RawConn) -> None:
        key = getattr(c, "pool_key", None) or (host, port, 0)
        lst = self.idle.setdefault(key, [])
        if len(lst) >= self.max_idle:
            c.close()
        else:
            c.idle_at = time.monotonic()
            lst.append(c)
        self.sweep()

    def sweep(self, force: bool = False) -> None:
        """Close connections idle longer than ``idle_s``, then the oldest
        ones beyond ``max_idle_total`` (checked at most every few seconds)."""
        now = time.monotonic()
        total = sum(len(v) for v in self.idle.values())
        if not force and now < self._next_sweep and total <= self.max_idle_total:
            return
        self._next_sweep = now + min(5.0, self.idle_s / 4)
        every = []
        for key, lst in list(self.idle.items()):
            keep = []
            for c in lst:
                if now - getattr(c, "idle_at", now) > self.idle_s:
                    c.close()
                else:
                    keep.append(c)
                    every.append((getattr(c, "idle_at", now), key, c))
            if keep:
                self.idle[key] = keep
            else:
                del self.idle[key]
        if len(every) > self.max_idle_total:
            every.sort(key=lambda t: t[0])
            for _t, key, c in every[:len(every) - self.max_idle_total]:
                self.idle[key].remove(c)
                if not self.idle[key]:
                    del self.idle[key]
                c.close()

    def close(self) -> None:
        for lst in self.idle.values():
            for c in lst:
                c.close()
        self.idle.clear()


async def _dial(host: str, port: int, timeout: float) -> socket.socket:
    """A connected non-blocking TCP socket: addresses raced with RFC 8305
    fast fallback (300 ms stagger, Go's net.Dialer default; utils/dial.py),
    ``timeout`` bounding the whole dial."""
    try:
        infos = await dial.resolve(host, port)
    except OSError as e:
        raise RawHTTPError(f"connect {host}:{port}: {e}") from e
    try:
        return await dial.connect_any(infos, timeout)
    except (OSError, asyncio.TimeoutError) as e:
        raise RawHTTPError(f"connect {host}:{port}: {e or type(e).__name__}") from e


def _hostport(host: str, port: int) -> str:
    return f"[{host}]:{port}" if ":" in host else f"{host}:{port}"


def proxy_auth_header(proxy) -> dict:
    """``{"Proxy-Authorization": ...}`` for absolute-form requests through an
    http(s) proxy with credentials, else {}."""
    if not absolute_form(proxy):
        return {}
    a = proxy.authorization()
    return {"Proxy-Authorization": a} if a else {}


async def _http_connect(c: RawConn, proxy, host: str, port: int, timeout: float) -> None:
    """``CONNECT host:port`` through an http proxy (Go's Transport: any
    status but 200 fails the dial with the status text)."""
    hp = _hostport(host, port)
    hdrs = {"Host": hp}
    if proxy.authorization():
        hdrs["Proxy-Authorization"] = proxy.authorization()
    await c.sendall(request_head("CONNECT", hp, hdrs), timeout)
    try:
        h = await read_head(c, timeout)
    except RawHTTPError as e:
        raise ProxyError(f"proxy {proxy.redacted()}: CONNECT {hp}: {e}") from e
    if h.status != 200:
        msg = f"proxy {proxy.redacted()} refused CONNECT {hp}: {h.status} {h.reason}"
        if h.status in (401, 403, 407):
            raise ProxyRefused(msg, h.status)
        raise ProxyError(msg)
    if h.leftover:
        raise ProxyError(f"proxy {proxy.redacted()}: data after the CONNECT reply")


async def _recv_exact(c: RawConn, n: int, timeout: float) -> bytes:
    buf = b""
    while len(buf) < n:
        d = await c.recv(n - len(buf), timeout)
        if not d:
            raise ProxyError("socks5 proxy closed the connection")
        buf += d
    return buf


_SOCKS_REPLIES = {1: "general failure", 2: "connection not allowed by ruleset", 3: "network unreachable",
                  4: "host unreachable", 5: "connection refused", 6: "TTL expired", 7: "command not supported",
                  8: "address type not supported"}


async def _socks5_connect(c: RawConn, proxy, host: str, port: int, timeout: float) -> None:
    """RFC 1928 CONNECT (RFC 1929 username/password when the proxy URL has
    userinfo — the methods Go's socks dialer offers); the target name is
    resolved by the proxy unless it is an IP literal."""
    import ipaddress
    import struct
    methods = b"\x00\x02" if proxy.username is not None else b"\x00"
    try:
        await c.sendall(b"\x05" + bytes([len(methods)]) + methods, timeout)
        ver, meth = await _recv_exact(c, 2, timeout)
        if ver != 5:
            raise ProxyError(f"socks5 proxy {proxy.redacted()}: unexpected protocol version {ver}")
        if meth == 0xFF:
            raise ProxyRefused(f"socks5 proxy {proxy.redacted()}: no acceptable authentication methods")
        if meth == 2:
            u, p = (proxy.username or "").encode(), (proxy.password or "").encode()
            await c.sendall(b"\x01" + bytes([len(u)]) + u + bytes([len(p)]) + p, timeout)
            _v, st = await _recv_exact(c, 2, timeout)
            if st != 0:
                raise ProxyRefused(f"socks5 proxy {proxy.redacted()}: username/password authentication failed")
        elif meth != 0:
            raise ProxyError(f"socks5 proxy {proxy.redacted()}: unsupported method {meth}")
        try:
            ip = ipaddress.ip_address(host)
            addr = (b"\x01" if ip.version == 4 else b"\x04") + ip.packed
        except ValueError:
            name = host.encode("idna")
            addr = b"\x03" + bytes([len(name)]) + name
        await c.sendall(b"\x05\x01\x00" + addr + struct.pack(">H", port), timeout)
        _v, rep, _r, atyp = await _recv_exact(c, 4, timeout)
        if rep != 0:
            msg = f"socks5 proxy {proxy.redacted()}: connect {_hostport(host, port)}: " \
                  f"{_SOCKS_REPLIES.get(rep, f'reply {rep}')}"
            raise (ProxyRefused(msg) if rep == 2 else ProxyError(msg))
        alen = {1: 4, 4: 16}.get(atyp)
        if alen is None:
            alen = (await _recv_exact(c, 1, timeout))[0]
        await _recv_exact(c, alen + 2, timeout)
    except asyncio.TimeoutError as e:
        raise ProxyError(f"socks5 proxy {proxy.redacted()}: handshake timed out") from e


_active_pumps = 0
_active_lock = __import__("threading").Lock()
_thread_time = __import__("time").thread_time


def active_pumps() -> int:
    """Relay pumps currently running in executor threads (tests / debugging)."""
    return _active_pumps


# thread CPU seconds and calls per relay pump (recv_body, send_body, ...) run
# on executor threads: the worker's CPU split by data-plane stage (bench diag)
PUMP_CPU: dict[str, list] = {}


def _counted(fn, *args):
    global _active_pumps
    with _active_lock:
        _active_pumps += 1
    t0 = _thread_time()
    try:
        return fn(*args)
    finally:
        dt = _thread_time() - t0
        name = getattr(fn, "__name__", "pump")
        with _active_lock:
            _active_pumps -= 1
            ent = PUMP_CPU.get(name)
            if ent is None:
                ent = PUMP_CPU[name] = [0.0, 0]
            ent[0] += dt
            ent[1] += 1


class _Port:
    """One event loop's ``_relay.CompletionPort``: relay pumps run on the
    native task pool and finish into it; the loop's reader on the port's
    eventfd resolves their futures (every pump finished since the last wake
    in one pass).  No interpreter thread is involved, unlike an executor
    hop (a Python thread wake-up, two GIL hand-offs and the loop's self-pipe
    per pump)."""

    def __init__(self, loop, relay) -> None:
        self.port = relay.CompletionPort()
        self.futs: dict[int, asyncio.Future] = {}
        self.next_id = 0
        self.start = {relay.recv_body: relay.start_recv_body, relay.send_body: relay.start_send_body}
        loop.add_reader(self.port.fileno(), self._drain)

    def _drain(self) -> None:
        global _active_pumps
        for pid, res in self.port.reap():
            fut = self.futs.pop(pid, None)
            with _active_lock:
                _active_pumps -= 1
            if fut is not None and not fut.done():
                fut.set_result(res)

    def submit(self, loop, fn, native, args) -> "asyncio.Future | None":
        start = self.start.get(fn)
        if start is None:
            return None
        global _active_pumps
        self.next_id += 1
        pid = self.next_id
        fut = loop.create_future()
        with _active_lock:
            _active_pumps += 1
        try:
            start(self.port, pid, native, *args)
        except BaseException:
            with _active_lock:
                _active_pumps -= 1
            raise
        self.futs[pid] = fut
        return fut


_ports: weakref.WeakKeyDictionary = weakref.WeakKeyDictionary()


def _native_pumps() -> bool:
    # opt-in: in isolation a port-started send pump is ~8 % faster than one on
    # an executor thread (profiles/r03_port_ab/upab), but whole headline jobs
    # measured slower on the box with it (profiles/r03_port_ab/SUMMARY.md)
    return os.environ.get("TRITONDL_RELAY_PORT", "0").lower() in ("1", "on", "true", "yes")


def _port(loop) -> "_Port | None":
    p = _ports.get(loop)
    if p is None:
        relay = relay_module()
        if relay is None or not hasattr(relay, "CompletionPort") or not _native_pumps():
            return None
        p = _ports[loop] = _Port(loop, relay)
    return p


async def run_pump(conn: RawConn, fn, *args):
    """Run a relay pump ``fn(conn.native, *args)`` in an executor thread, or
    with ``TRITONDL_RELAY_PORT=1`` (``recv_body`` / ``send_body``) on the
    native task pool through the loop's completion port.

    If the awaiting task is cancelled, the pump is aborted (sticky native flag
    + socket shutdown, fd left open) and awaited to completion before the
    cancellation propagates — so the caller's ``finally`` can never close a
    socket or file the pump is still using (fd numbers are reused)."""
    loop = asyncio.get_running_loop()
    port = _port(loop)
    fut = port.submit(loop, fn, conn.native, args) if port is not None else None
    if fut is None:
        fut = loop.run_in_executor(None, _counted, fn, conn.native, *args)
    try:
        return await asyncio.shield(fut)
    except asyncio.CancelledError:
        conn.abort()
        while not fut.done():
            try:
                await asyncio.shield(fut)
            except asyncio.CancelledError:
                continue
            except Exception:  # noqa: BLE001 - the pump's own error no longer matters
                break
        raise


async def run_settled(loop, fn, *args):
    """``fn(*args)`` in an executor thread, awaited to completion even if the
    caller is cancelled (the cancellation is re-raised once it returned).
    For blocking I/O on a descriptor the caller closes afterwards: a write
    still running in the thread when the fd is closed and its number reused
    would land in whatever file took the number."""
    fut = loop.run_in_executor(None, fn, *args)
    try:
        return await asyncio.shield(fut)
    except asyncio.CancelledError:
        while not fut.done():
            try:
                await asyncio.shield(fut)
            except asyncio.CancelledError:
                continue
            except Exception:  # noqa: BLE001 - the write's own error no longer matters
                break
        raise


_client_tls: dict = {}


def client_tls_context(ca_file: str = "", verify: bool = True):
    """Shared client ``_relay.TlsContext`` (one per CA setting, so session
    tickets are reused across connections).  ``ca_file`` "" = the system
    store; ``SSL_CERT_FILE`` is honoured, and ``TRITONDL_CA_FILE`` names an
    extra trust file (e.g. a private MinIO CA)."""
    relay = relay_module()
    if relay is None:
        return None
    ca_file = ca_file or os.environ.get("TRITONDL_CA_FILE", "")
    key = (ca_file, verify)
    ctx = _client_tls.get(key)
    if ctx is None:
        ctx = _client_tls[key] = relay.TlsContext.client(ca_file=ca_file, verify=verify)
    return ctx


def request_head(method: str, target: str, headers: dict) -> bytes:
    lines = [f"{method} {target} HTTP/1.1"]
    lines += [f"{k}: {v}" for k, v in headers.items()]
    return ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1")


async def _recv(s, n: int, timeout: float) -> bytes:
    if isinstance(s, RawConn):
        return await s.recv(n, timeout)
    return await asyncio.wait_for(asyncio.get_running_loop().sock_recv(s, n), timeout)


async def read_head(s: "RawConn | socket.socket", timeout: float, max_size: int = 64 << 10) -> Head:
    buf = b""
    while True:
        i = buf.find(b"\r\n\r\n")
        if i >= 0:
            break
        if len(buf) > max_size:
            raise RawHTTPError("response head too large")
        try:
            d = await _recv(s, 256 << 10, timeout)
        except asyncio.TimeoutError as e:
            raise RawHTTPError("timed out waiting for the response head") from e
        if not d:
            raise RawHTTPError("connection closed before the response head")
        buf += d
    return parse_head(buf[:i], buf[i + 4:])


def parse_head(raw: bytes, leftover: bytes = b"") -> Head:
    """Status line and header fields of a response head (``raw`` without its
    blank line); a malformed status line or Content-Length is a RawHTTPError."""
    lines = raw.decode("latin-1").split("\r\n")
    ver, _, rest = lines[0].partition(" ")
    code, _, reason = rest.partition(" ")
    if not ver.startswith("HTTP/") or not (len(code) == 3 and code.isascii() and code.isdigit()):
        raise RawHTTPError(f"malformed status line {lines[0]!r}")
    hdrs: CIMultiDict = CIMultiDict()
    for ln in lines[1:]:
        k, sep, v = ln.partition(":")
        if sep:
            hdrs.add(k.strip(), v.strip())
    conn = hdrs.get("Connection", "").lower()
    keep = (ver == "HTTP/1.1" and conn != "close") or conn == "keep-alive"
    chunked = "chunked" in hdrs.get("Transfer-Encoding", "").lower()
    if keep and "Content-Length" in hdrs and chunked:
        keep = False            # ambiguous framing (RFC 9112 §6.3): never reuse this connection
    if not chunked and "Content-Length" in hdrs:
        cls = {x.strip() for v in hdrs.getall("Content-Length") for x in v.split(",")}   # "42, 42" is 42
        if len(cls) != 1 or not all(v.isascii() and v.isdigit() for v in cls):
            raise RawHTTPError(f"bad Content-Length {hdrs.getall('Content-Length')!r}")   # RFC 9112 §6.3
    return Head(int(code), reason, hdrs, leftover, ver, keep)


_HEX = frozenset(b"0123456789abcdefABCDEF")


def _chunk_size(line: bytes) -> int:
    """RFC 9112 §7.1 chunk-size (hex digits, optional ``;ext``).  Anything
    else — a sign, ``0x``, spaces, an empty or over-long size — is a
    RawHTTPError: ``int(x, 16)`` took "-5", whose negative length then moved
    the parser backwards over the same line forever."""
    size = line.split(b";", 1)[0].rstrip(b" \t")
    if not size or len(size) > 16 or not all(c in _HEX for c in size):
        raise RawHTTPError(f"bad chunk size {line[:40]!r}")
    return int(size, 16)


async def read_small_body(s: "RawConn | socket.socket", head: Head, timeout: float, limit: int = 16 << 20,
                          method: str = "GET") -> bytes:
    """Whole body of a small response (Content-Length, chunked, or until
    close).  Marks ``head.keep_alive`` False when the connection can't be
    reused."""
    buf = bytearray(head.leftover)

    async def more() -> bool:
        try:
            d = await _recv(s, 256 << 10, timeout)
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
            n = _chunk_size(bytes(buf[pos:j]))
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
