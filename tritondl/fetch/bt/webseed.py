"""BEP 19 web seeds ("GetRight style" ``url-list`` / magnet ``ws=``).

anacrolix/torrent, which the reference embeds (SURVEY.md §2.1 C7,
``internal/downloader/torrent/torrent.go:18-119``), fetches pieces from a
torrent's web seeds alongside the swarm; this is the equivalent.  Each web
seed runs ``conns`` workers; a worker claims a whole piece nobody is fetching
(preferring pieces no connected peer has), fetches the byte spans the piece
covers with HTTP Range requests — one per file the piece straddles — and hands
the bytes to :meth:`Torrent.commit_piece`, the same verify → write → announce
path peer downloads use.  HTTP failures back off exponentially; a seed that
serves ``max_bad`` pieces failing the hash check is dropped.
"""

from __future__ import annotations

import asyncio
import contextlib
from typing import TYPE_CHECKING
from urllib.parse import quote

import aiohttp

from ...utils.dial import FALLBACK_DELAY, socket_factory
from ...utils.log import log

if TYPE_CHECKING:  # pragma: no cover
    from .torrent import Torrent


# a web seed answering Range with 200 is streamed past at most this many bytes per span
IGNORED_RANGE_MAX_SKIP = 64 << 20


async def _read_span(r: aiohttp.ClientResponse, skip: int, n: int) -> bytes:
    """``n`` bytes of the body after the first ``skip``; never holds more
    than ``n`` bytes, whatever the server sends (an over-long body is left
    unread and its connection closed)."""
    while skip > 0:
        chunk = await r.content.read(min(skip, 1 << 20))
        if not chunk:
            return b""
        skip -= len(chunk)
    out = bytearray()
    while len(out) < n:
        chunk = await r.content.read(min(n - len(out), 1 << 20))
        if not chunk:
            break
        out += chunk
    return bytes(out)


class WebSeedError(Exception):
    pass


def file_url(base: str, name: str, path: list[str], multi: bool) -> str:
    """BEP 19 URL of one torrent file under web seed ``base``."""
    if not multi:
        return base + quote(name) if base.endswith("/") else base
    if not base.endswith("/"):
        base += "/"
    return base + "/".join(quote(c) for c in [name, *path])


class WebSeed:
    def __init__(self, t: "Torrent", url: str, conns: int = 4, max_bad: int = 3,
                 session: aiohttp.ClientSession | None = None) -> None:
        self.t = t
        self.url = url
        self.conns = max(1, conns)
        self.max_bad = max_bad
        self._session = session
        self.bad = 0
        self.pieces_ok = 0
        self.bytes = 0
        self.dead = False
        self._cursor = 0

    async def run(self) -> None:
        await self.t.got_info.wait()
        while not self.t.closed and not self.t._downloading:
            await asyncio.sleep(0.05)
        own = self._session is None
        session = self._session or aiohttp.ClientSession(
            timeout=aiohttp.ClientTimeout(total=None, sock_connect=15, sock_read=60),
            connector=aiohttp.TCPConnector(limit=self.conns, force_close=False,
                                           happy_eyeballs_delay=FALLBACK_DELAY, socket_factory=socket_factory))
        try:
            await asyncio.gather(*(self._worker(session) for _ in range(self.conns)))
        finally:
            if own:
                await session.close()

    # -- piece choice --------------------------------------------------------
    def _claim(self) -> int | None:
        t = self.t
        info = t.info
        assert info is not None
        n = info.num_pieces
        fallback = None
        for k in range(n):
            i = (self._cursor + k) % n
            if t.have[i] or t.in_flight(i) or i in t.ws_busy:
                continue
            if t.avail[i] == 0:          # nobody in the swarm has it: ours
                self._cursor = i + 1
                t.ws_busy.add(i)
                return i
            if fallback is None:
                fallback = i
        if fallback is not None and not t.peers:
            t.ws_busy.add(fallback)
            self._cursor = fallback + 1
            return fallback
        if fallback is not None and len(t.peers) < 2:
            # thin swarm: help with pieces peers have too
            t.ws_busy.add(fallback)
            self._cursor = fallback + 1
            return fallback
        return None

    # -- fetching ------------------------------------------------------------
    def _spans(self, i: int) -> list[tuple[str, int, int]]:
        info = self.t.info
        assert info is not None
        start = i * info.piece_length
        end = start + info.piece_size(i)
        out = []
        for f in info.files:
            fs, fe = f.offset, f.offset + f.length
            if fe <= start or fs >= end or f.length == 0:
                continue
            a, b = max(start, fs), min(end, fe)
            # BEP 47 padding is never served: an empty URL means zeros
            out.append(("" if f.pad else file_url(self.url, info.name, f.path, info.multi), a - fs, b - a))
        return out

    async def _fetch(self, session: aiohttp.ClientSession, i: int) -> bytearray:
        buf = bytearray()
        for url, off, n in self._spans(i):
            if not url:
                buf += bytes(n)
                continue
            hdr = {"Range": f"bytes={off}-{off + n - 1}"}
            async with session.get(url, headers=hdr) as r:
                if r.status == 206:
                    data = await _read_span(r, 0, n)
                elif r.status == 200:
                    # server ignored Range: take our slice of the full body, streaming
                    # past the bytes before it; a seed that would make every piece
                    # stream a large prefix is dropped (never buffered whole)
                    if off > IGNORED_RANGE_MAX_SKIP:
                        self.dead = True
                        raise WebSeedError(f"{url} ignores Range requests; dropping the web seed")
                    data = await _read_span(r, off, n)
                else:
                    raise WebSeedError(f"HTTP {r.status} for {url}")
            if len(data) != n:
                raise WebSeedError(f"short read from {url}: {len(data)} != {n}")
            buf += data
        return buf

    async def _worker(self, session: aiohttp.ClientSession) -> None:
        t = self.t
        backoff = 0.5
        while not t.closed and not t.complete.is_set() and not self.dead:
            i = self._claim()
            if i is None:
                await asyncio.sleep(0.2)
                continue
            try:
                data = await self._fetch(session, i)
                ok = await t.commit_piece(i, data)
            except (aiohttp.ClientError, asyncio.TimeoutError, WebSeedError, OSError) as e:
                log.with_fields(webseed=self.url, piece=i, error=str(e) or type(e).__name__).debug("web seed fetch failed")
                t.ws_busy.discard(i)
                await asyncio.sleep(backoff)
                backoff = min(backoff * 2, 60.0)
                continue
            finally:
                with contextlib.suppress(KeyError):
                    t.ws_busy.remove(i)
            backoff = 0.5
            if ok:
                self.pieces_ok += 1
                self.bytes += len(data)
            elif ok is None:
                await asyncio.sleep(0.2)     # v2 piece layer not known yet: not the seed's fault
            else:
                self.bad += 1
                log.with_fields(webseed=self.url, piece=i).warn("web seed piece failed hash check")
                if self.bad >= self.max_bad:
                    log.with_field("webseed", self.url).warn("dropping web seed: too many bad pieces")
                    self.dead = True
