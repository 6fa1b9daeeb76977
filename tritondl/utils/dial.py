"""Outbound TCP dials with RFC 6555 / RFC 8305 fast fallback ("Happy Eyeballs").

Every dial in the reference went through Go's ``net.Dialer``, whose zero
value (Go >= 1.12) races the address families of a dual-stack name: the
first family is tried, and 300 ms later (``FallbackDelay``) the other family
joins the race; the first connection wins.  That covers grab's transport
(``internal/downloader/http/http.go:18-22``), minio-go's
(``internal/uploader/uploader.go:43-51``) and ``amqp.Dial``
(``internal/rabbitmq/client.go:308-309``).  A node whose AAAA answers are
black-holed therefore lost 300 ms per connection there, not a full connect
timeout.

:func:`dial` does the same for this worker's native data plane (HTTP GET
and S3 PUT pumps, :mod:`tritondl.utils.rawhttp`), the AMQP connection and
BitTorrent TCP peers.  It follows RFC 8305 §4-5, the generalisation of Go's
two-family race: resolved addresses are interleaved by family (first
family first), a new attempt starts every ``delay`` seconds or as soon as
the previous one fails, attempts overlap, and the first socket to connect
wins; the others are cancelled and closed.  ``timeout`` bounds the whole
dial, not each attempt.

Every dialed socket also gets Go's default TCP keep-alive (:func:`keepalive`):
a zero-value ``net.Dialer`` (and ``net.ListenConfig`` for accepted sockets)
enables it with 15 s idle and 15 s between probes.  A pooled keep-alive
connection, an AMQP connection between heartbeats or a PUT waiting on its
download that crosses a NAT or conntrack table with an idle timeout stays
mapped, and a dead peer is noticed in ~2.5 min instead of at the next
200-300 s application timeout.  The aiohttp connectors get the same through
:func:`socket_factory`.
"""

from __future__ import annotations

import asyncio
import socket

FALLBACK_DELAY = 0.3            # Go net.Dialer: "If zero, a default delay of 300ms is used"
KEEPALIVE_IDLE = 15             # Go net.Dialer.KeepAlive zero value: probes after 15 s idle ...
KEEPALIVE_INTERVAL = 15         # ... every 15 s ...
KEEPALIVE_COUNT = 9             # ... 9 unanswered probes (Go's KeepAliveConfig default, Linux's too)


def keepalive(s: socket.socket, idle: int = KEEPALIVE_IDLE, interval: int = KEEPALIVE_INTERVAL,
              count: int = KEEPALIVE_COUNT) -> None:
    """TCP keep-alive as Go's net.Dialer sets it (``SO_KEEPALIVE`` plus
    ``TCP_KEEPIDLE`` / ``TCP_KEEPINTVL`` / ``TCP_KEEPCNT`` where the OS has them)."""
    s.setsockopt(socket.SOL_SOCKET, socket.SO_KEEPALIVE, 1)
    for opt, v in (("TCP_KEEPIDLE", idle), ("TCP_KEEPINTVL", interval), ("TCP_KEEPCNT", count)):
        if hasattr(socket, opt):
            s.setsockopt(socket.IPPROTO_TCP, getattr(socket, opt), int(v))


def tcp_options(s: socket.socket) -> None:
    """Options of every TCP socket this worker dials or accepts."""
    if s.family in (socket.AF_INET, socket.AF_INET6) and s.type == socket.SOCK_STREAM:
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        keepalive(s)


def socket_factory(addr_info) -> socket.socket:
    """aiohttp ``TCPConnector(socket_factory=...)``: its sockets get the same
    options as :func:`dial`'s."""
    fam, typ, proto, _cn, _addr = addr_info
    s = socket.socket(fam, typ, proto)
    try:
        tcp_options(s)
    except OSError:
        s.close()
        raise
    return s


def interleave(infos: list) -> list:
    """RFC 8305 §4: alternate address families, starting with the family of
    the first address (``getaddrinfo`` has already sorted by RFC 6724)."""
    if not infos:
        return []
    first = infos[0][0]
    a = [i for i in infos if i[0] == first]
    b = [i for i in infos if i[0] != first]
    out = []
    for k in range(max(len(a), len(b))):
        if k < len(a):
            out.append(a[k])
        if k < len(b):
            out.append(b[k])
    return out


async def _attempt(loop: asyncio.AbstractEventLoop, info) -> socket.socket:
    fam, typ, proto, _cn, addr = info
    s = socket.socket(fam, typ, proto)
    try:
        s.setblocking(False)
        tcp_options(s)
        await loop.sock_connect(s, addr)
    except BaseException:
        s.close()
        raise
    return s


async def connect_any(infos: list, timeout: float, delay: float = FALLBACK_DELAY) -> socket.socket:
    """Staggered race over resolved ``getaddrinfo`` entries; returns the first
    connected non-blocking socket.  Raises the last connect error, or
    :class:`TimeoutError` once ``timeout`` has passed."""
    loop = asyncio.get_running_loop()
    order = interleave(list(infos))
    if not order:
        raise OSError("no addresses to dial")
    deadline = loop.time() + timeout
    pending: set[asyncio.Future] = set()
    last_err: BaseException | None = None
    nxt = 0
    try:
        while True:
            if nxt < len(order):
                pending.add(asyncio.ensure_future(_attempt(loop, order[nxt])))
                nxt += 1
            left = deadline - loop.time()
            if left <= 0:
                raise TimeoutError(f"dial timed out after {timeout:.1f}s")
            # wait for a result, or for the stagger delay to start the next address
            wait = min(delay, left) if nxt < len(order) else left
            done, pending = await asyncio.wait(pending, timeout=wait, return_when=asyncio.FIRST_COMPLETED)
            won: socket.socket | None = None
            for t in done:
                if t.cancelled():
                    continue
                e = t.exception()
                if e is not None:
                    last_err = e
                elif won is None:
                    won = t.result()
                else:
                    t.result().close()          # two connected in the same tick: keep one
            if won is not None:
                return won
            if not pending and nxt >= len(order):
                raise last_err if last_err is not None else OSError("dial failed")
            # a failure starts the next attempt at once (RFC 8305 §5); a timeout is the stagger
    finally:
        for t in pending:
            t.cancel()
        if pending:
            res = await asyncio.gather(*pending, return_exceptions=True)
            for r in res:
                if isinstance(r, socket.socket):
                    r.close()


def literal_infos(host: str, port: int) -> list | None:
    """``getaddrinfo``-shaped entries for an IP literal (no resolver thread hop,
    as asyncio's own fast path), else None."""
    import ipaddress
    try:
        ip = ipaddress.ip_address(host.strip("[]"))
    except ValueError:
        return None
    fam = socket.AF_INET6 if ip.version == 6 else socket.AF_INET
    addr = (str(ip), port, 0, 0) if ip.version == 6 else (str(ip), port)
    return [(fam, socket.SOCK_STREAM, socket.IPPROTO_TCP, "", addr)]


async def resolve(host: str, port: int) -> list:
    infos = literal_infos(host, port)
    if infos is None:
        infos = await asyncio.get_running_loop().getaddrinfo(host, port, type=socket.SOCK_STREAM)
    return infos


async def dial(host: str, port: int, timeout: float = 30.0, delay: float = FALLBACK_DELAY) -> socket.socket:
    """Resolve ``host`` and connect with fast fallback; a connected
    non-blocking TCP socket (``TCP_NODELAY`` and keep-alive set)."""
    return await connect_any(await resolve(host, port), timeout, delay)


async def open_connection(host: str, port: int, *, timeout: float = 30.0, delay: float = FALLBACK_DELAY,
                          ssl=None, **kw) -> tuple[asyncio.StreamReader, asyncio.StreamWriter]:
    """``asyncio.open_connection`` over a fast-fallback dial (TLS, if any,
    verifies ``host``)."""
    s = await dial(host, port, timeout, delay)
    try:
        if ssl is not None:
            kw.setdefault("server_hostname", host)
        return await asyncio.open_connection(sock=s, ssl=ssl, **kw)
    except BaseException:
        s.close()
        raise


__all__ = ["FALLBACK_DELAY", "keepalive", "tcp_options", "socket_factory", "interleave", "connect_any", "literal_infos", "resolve", "dial", "open_connection"]
