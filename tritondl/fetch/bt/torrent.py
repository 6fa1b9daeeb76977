"""One torrent's swarm session: peer discovery, metadata exchange, piece
picking, block pipelining, verification, storage and seeding.

This is the capability of the ~10 anacrolix/torrent calls the reference makes
(``internal/downloader/torrent/torrent.go:40-106``: NewClient with file
storage, AddMagnet, GotInfo, DownloadAll, BytesCompleted, Info().TotalLength,
WaitAll, Close), implemented from the BEPs:

* discovery: magnet ``x.pe`` peers, every tracker (HTTP / UDP), the DHT
  (``get_peers`` + ``announce_peer``), and inbound connections on our
  listen port;
* metadata (magnet → info dict) over ut_metadata, verified against the
  info-hash;
* rarest-first piece picking with an end-game mode; up to ``pipeline``
  outstanding 16 KiB block requests per unchoked peer;
* every completed piece is SHA-1 verified (worker thread) before it is
  written and announced with HAVE; peers sending bad data are dropped;
* we serve requests from interested peers while downloading (and after, if
  ``seed``), like anacrolix's default client;
* resume: existing data is batch-verified at start (HIP kernel when a GPU
  helps, see :mod:`.storage`), so a redelivered job continues.
"""

from __future__ import annotations

import asyncio
import collections
import contextlib
import errno
import functools
import hashlib
import heapq
import itertools
import os
import random
import socket
import struct
import time
from dataclasses import dataclass, field

from ...ops import hashing
from ...utils import dial as tcpdial
from ...utils.disk import check_space
from ...utils.log import log
from . import bep40, merkle, mse
from . import peer as pw
from .dht import DHTNode
from .metainfo import BLOCK, Info, MetainfoError
from .storage import CompletionDB, FileStorage
from .tracker import Announce, TrackerError, announce, new_peer_id

try:  # native peer-wire data plane (csrc/btwire): block assembly + request pipelining
    from ... import _btwire as _W  # type: ignore[attr-defined]
except ImportError:  # pragma: no cover - the extension ships with every build
    _W = None

# Live v1 verification: completed pieces per executor hop.  16 when the host
# has the 16-lane AVX-512 SHA-1 (hash_core.h md_batch; a partial group waits
# at most VERIFY_WAIT_S for partners), else an SHA-NI pair.
VERIFY_GROUP = 16 if hashing.sha_mb() else 2
VERIFY_WAIT_S = 0.003


@dataclass
class TorrentConfig:
    # anacrolix NewDefaultClientConfig (torrent.go:40): EstablishedConnsPerTorrent 50,
    # HalfOpenConnsPerTorrent 25 — peers with a finished handshake, and dials in flight
    established_conns: int = 50
    half_open_conns: int = 25
    # anacrolix TorrentPeersHighWater: addresses remembered per torrent (trackers,
    # DHT, PEX); past it a new one replaces an unconnected one
    peers_high_water: int = 500
    pipeline: int = 128
    listen_host: str = "0.0.0.0"
    listen_port: int = 0             # 0 = ephemeral (the worker's Config passes anacrolix's 42069)
    listen_port_fallback: bool = True  # listen_port busy (another torrent / worker has it): use an ephemeral one
    announce_host: str | None = None
    seed: bool = False
    request_timeout: float = 20.0
    connect_timeout: float = 5.0
    verify_device: str = "auto"
    tracker_min_interval: float = 30.0
    dht_interval: float = 60.0
    utp: bool = False
    pex: bool = True                 # BEP 11 peer exchange (off for private torrents regardless)
    pex_interval: float = 60.0
    webseed_conns: int = 4           # BEP 19: concurrent piece fetches per web seed
    encryption: str = "allow"        # MSE/PE policy: disable | allow | prefer | require (see .mse)
    layer_timeout: float = 120.0     # BEP 52: time to fetch piece layers of a v2 magnet
    upnp: bool = False               # forward the listen port (TCP+UDP) via a UPnP gateway (see .portfwd)
    upnp_ssdp: tuple | None = None   # SSDP target (default: the 239.255.255.250:1900 multicast group)
    disk_reserve: int = 0            # bytes to keep free on the job's filesystem (utils.disk preflight)
    listen_host6: str | None = None  # also accept peers on IPv6 (same port), e.g. "::"
    native_wire: bool = True         # per-block work in csrc/btwire (False: the pure-Python path)


def _block_digest(piece, b: int) -> bytes:
    """Short digest of block ``b`` of a piece buffer (smart-ban evidence)."""
    return hashlib.sha1(piece[b * BLOCK:(b + 1) * BLOCK]).digest()[:12]


@dataclass
class _Piece:
    size: int
    nblocks: int
    buf: bytearray
    received: set = field(default_factory=set)            # block indexes
    requested: dict = field(default_factory=dict)          # block idx -> set(peer keys)
    next_b: int = 0                                        # blocks < next_b were handed out once
    redo: list = field(default_factory=list)               # handed-out blocks whose requests all lapsed
    src: dict = field(default_factory=dict)                # block idx -> key of the peer that supplied it

    def take(self) -> int | None:
        """Next never-requested (or lapsed) block; O(1) amortised instead of a
        per-call scan over every block (the scan was half the leecher's CPU)."""
        while self.redo:
            b = self.redo.pop()
            if b not in self.received and b not in self.requested:
                return b
        if self.next_b < self.nblocks:
            self.next_b += 1
            return self.next_b - 1
        return None

    def lapse(self, b: int, key) -> bool:
        """Drop key's request for block b; True if b became requestable again."""
        s = self.requested.get(b)
        if s is not None:
            s.discard(key)
            if not s:
                del self.requested[b]
                if b not in self.received:
                    self.redo.append(b)
                    return True
        return False


class _Peer:
    def __init__(self, wire: pw.Wire, addr: tuple[str, int], hs: pw.Handshake, n: int) -> None:
        self.wire = wire
        self.addr = addr
        self.hs = hs
        self.key = addr
        self.have = bytearray(n)
        self.nhave = 0
        self.peer_choking = True
        self.peer_interested = False
        self.am_interested = False
        self.ext: pw.ExtHandshake | None = None
        self.outstanding: dict[tuple[int, int], float] = {}
        self.listen_addr: tuple[str, int] | None = None   # where others can dial it (PEX)
        self.pex_sent: set[tuple[str, int]] = set()
        self.bad = 0                                        # failed pieces it supplied blocks of
        self.good = 0                                       # verified pieces it supplied blocks of
        self.lid = 0                                        # its native link's id (PieceStore blame)
        self.wants = 0                                      # pieces it has that we lack
        self.downloaded = 0
        self.meta_requested = False
        self.meta_asked_at = 0.0
        self.link = None                                    # _btwire.Link once the native data plane runs
        self.rx: pw.LinkReader | None = None                # zero-copy receive into the link (plain TCP)
        self.rx_tried = False
        # requests withdrawn (lapsed / cancelled) lately: a block that answers one is
        # still accepted; a block matching neither this nor `outstanding` is dropped
        self.recent: dict[tuple[int, int], int] = {}
        self.wasted = 0

    def withdrew(self, k: tuple[int, int]) -> None:
        self.recent[k] = 1
        if len(self.recent) > 1024:
            del self.recent[next(iter(self.recent))]

    def set_have(self, i: int) -> bool:
        if 0 <= i < len(self.have) and not self.have[i]:
            self.have[i] = 1
            self.nhave += 1
            return True
        return False


class Torrent:
    def __init__(self, infohash: bytes, base_dir: str, cfg: TorrentConfig | None = None, *,
                 info: Info | None = None, trackers: list[str] | None = None,
                 peers: list[tuple[str, int]] | None = None, dht: DHTNode | None = None,
                 peer_id: bytes | None = None, name_hint: str = "",
                 webseeds: list[str] | None = None) -> None:
        self.infohash = infohash
        self.base_dir = base_dir
        self.cfg = cfg or TorrentConfig()
        self.trackers = list(trackers or [])
        self.static_peers = list(peers or [])
        self.webseeds = list(dict.fromkeys(webseeds or []))
        self.ws_busy: set[int] = set()                  # pieces a web seed is fetching
        self.webseed_clients: list = []
        self.pex_learned = 0
        self.dht = dht
        self.peer_id = peer_id or new_peer_id()
        self.name_hint = name_hint
        self.info: Info | None = None
        self.storage: FileStorage | None = None
        self.db: CompletionDB | None = None
        self.have = bytearray()
        self.nhave = 0
        self.avail: list[int] = []
        self.pieces: dict[int, _Piece] = {}
        self.open_pieces: dict[int, _Piece] = {}        # subset of pieces with blocks left to hand out
        self.verifying: set[int] = set()                # complete pieces being hashed/written
        self._layer_waiters: dict = {}                  # (root, index, peer) -> future of a v2 hashes reply
        self._rare: list[int] | None = None             # missing pieces by availability (picker order)
        self._rare_pos = 0
        self._rare_t = 0.0
        self._rare_dirty = True
        self._finishers: set[asyncio.Task] = set()
        self.store = None                               # _btwire.PieceStore (native data plane)
        self._my_ip: str | None = None                  # learned from our first connection
        self._prio: dict[tuple[str, int], int] = {}     # BEP 40 priority cache
        self.source = None                              # _btwire.Source: links serve REQUESTs from it
        self.fatal: BaseException | None = None         # storage error that ends the download
        self.failed = asyncio.Event()
        self._vq: list = []                             # (piece, data, peer) awaiting a verify partner
        self._vflush = False
        self.assigned: dict[int, set] = {}              # piece -> peer keys whose links fetch it
        # per-file completion (streamed uploads): see watch_files
        self._file_cb = None                            # callable(path) for watched files
        self._file_pick = None                          # callable([paths]) -> set of paths to watch
        self._file_left: dict[int, int] = {}            # watched file index -> pieces still missing
        self._piece_files: dict[int, list[int]] = {}    # piece -> watched files it covers
        self._piece_rank: list[int] | None = None       # picker band per piece (lower first)
        self.peers: dict[tuple[str, int], _Peer] = {}
        self.known: set[tuple[str, int]] = set()
        self.connecting: set[tuple[str, int]] = set()
        self.banned: set[tuple[str, int]] = set()
        # (good, bad) pieces each peer address supplied blocks of: anacrolix's
        # netGoodPiecesDirtied, outliving a connection so a reconnect keeps its record
        self.trust: dict[tuple[str, int], list[int]] = {}
        self._lid_key: dict[int, tuple[str, int]] = {}  # native link id -> peer key
        self._lids = itertools.count(1)
        # failed pieces: (block, peer key, block digest) of what each peer sent, checked
        # against the data once the piece verifies (smart ban); and the one peer a piece
        # whose blame was a tie is re-fetched from
        self._failed_blocks: dict[int, list[tuple[int, tuple, bytes]]] = {}
        self._isolate: dict[int, tuple[str, int]] = {}
        self.got_info = asyncio.Event()
        self.complete = asyncio.Event()
        self._downloading = False
        self._meta_size: int | None = None
        self._meta: dict[int, bytes] = {}
        # BEP 9 metadata from untrusted peers: which peer sent each piece, peers whose
        # metadata failed the info-hash (never asked again), and one-source mode after a
        # failure with several contributors (the next failure then names its culprit)
        self._meta_src: dict[int, tuple] = {}
        self._meta_bad: set = set()
        self._meta_single = False
        self._tasks: set[asyncio.Task] = set()
        self._server: asyncio.AbstractServer | None = None
        self._server6: asyncio.AbstractServer | None = None
        self.port = 0
        self.utp = None
        self.portfwd = None
        self._uploaded = 0                              # Python-served bytes + links of dropped peers
        self.downloaded = 0
        self.wasted = 0                                 # unrequested block bytes dropped (Python wire)
        self.closed = False
        self._wake = asyncio.Event()
        if info is not None:
            self._set_info(info)

    # ------------------------------------------------------------ lifecycle
    def _spawn(self, coro) -> asyncio.Task:
        t = asyncio.ensure_future(coro)
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)
        return t

    async def _listen(self, port: int) -> None:
        self._server = await asyncio.start_server(self._on_inbound, self.cfg.listen_host, port)
        self.port = self._server.sockets[0].getsockname()[1]

    async def start(self) -> None:
        try:
            await self._listen(self.cfg.listen_port)
        except OSError as e:
            # anacrolix fails NewClient on a busy port; here one worker process can run
            # several torrents (and a node several workers), so the later ones take an
            # ephemeral port instead (announced to trackers / the DHT as usual)
            if not (self.cfg.listen_port and self.cfg.listen_port_fallback and e.errno == errno.EADDRINUSE):
                raise
            log.with_fields(port=self.cfg.listen_port).info("bittorrent listen port busy; using an ephemeral port")
            await self._listen(0)
        if self.cfg.utp:
            from .utp import UtpSocket
            # uTP shares the TCP port number, as anacrolix/libutp do.  A port the
            # kernel picked for TCP can be taken on UDP (a DHT node, another
            # worker's uTP): then move both to another ephemeral port, as
            # anacrolix's listenAll retries, instead of running without uTP
            for attempt in range(16):
                try:
                    self.utp = await UtpSocket().start(self.cfg.listen_host, self.port)
                    self._spawn(self._utp_accept_loop())
                    break
                except OSError as e:
                    self.utp = None
                    movable = e.errno == errno.EADDRINUSE and (not self.cfg.listen_port or
                                                               self.cfg.listen_port_fallback)
                    if not movable or attempt == 15:
                        log.with_field("error", str(e)).warn("uTP disabled: cannot bind UDP port")
                        break
                    log.with_fields(port=self.port).debug("UDP port busy; moving to another port pair")
                    self._server.close()
                    await self._server.wait_closed()
                    await self._listen(0)
        if self.cfg.listen_host6 is not None:
            # dual stack like anacrolix: the same port on IPv6, so peers learnt from the
            # IPv6 DHT / PEX (announced with this port) can dial in
            try:
                s6 = socket.socket(socket.AF_INET6, socket.SOCK_STREAM)
                s6.setsockopt(socket.IPPROTO_IPV6, socket.IPV6_V6ONLY, 1)
                s6.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                s6.bind((self.cfg.listen_host6, self.port))
                self._server6 = await asyncio.start_server(self._on_inbound, sock=s6)
            except OSError as e:
                log.with_field("error", str(e)).debug("IPv6 listen socket unavailable")
                self._server6 = None
        if self.cfg.upnp:
            from .portfwd import SSDP_ADDR, PortForwarder
            self.portfwd = PortForwarder(self.port, ssdp_addr=self.cfg.upnp_ssdp or SSDP_ADDR)
            self._spawn(self.portfwd.start())      # discovery runs in the background, never on the job path
        for p in self.static_peers:
            self.add_peer_addr(p)
        for url in self.trackers:
            self._spawn(self._tracker_loop(url))
        if self.dht is not None:
            self._spawn(self._dht_loop())
        self._spawn(self._timeout_loop())
        if self.cfg.pex:
            self._spawn(self._pex_loop())
        if self.webseeds:
            from .webseed import WebSeed
            for url in self.webseeds:
                ws = WebSeed(self, url, self.cfg.webseed_conns)
                self.webseed_clients.append(ws)
                self._spawn(ws.run())

    async def _utp_accept_loop(self) -> None:
        assert self.utp is not None
        while not self.closed:
            r, w, _addr = await self.utp.accept()
            self._spawn(self._on_inbound(r, w))

    async def close(self) -> None:
        if self.closed:
            return
        self.closed = True
        if self._server is not None:
            self._server.close()
        if self._server6 is not None:
            self._server6.close()
        if self.utp is not None:
            self.utp.close()
        for p in list(self.peers.values()):
            p.wire.close()
        for t in list(self._tasks):
            t.cancel()
        for t in list(self._tasks):
            with contextlib.suppress(BaseException):
                await t
        for t in list(self._finishers):   # executor hash/write jobs must land before storage closes
            with contextlib.suppress(BaseException):
                await t
        if self.source is not None:
            self.source.close()           # links stop serving before the job's files go away
        if self.storage is not None:
            self.storage.close()
        if self.db is not None:
            self.db.close()
        if self.portfwd is not None:
            with contextlib.suppress(Exception):
                await asyncio.wait_for(self.portfwd.close(), 5.0)
        if self._server is not None:
            with contextlib.suppress(Exception):
                await self._server.wait_closed()

    # ------------------------------------------------------------ info / storage
    def _set_info(self, info: Info) -> None:
        if not info.matches(self.infohash):
            raise MetainfoError("info dict does not match info-hash")
        self.info = info
        n = info.num_pieces
        self.have = bytearray(n)
        self.avail = [0] * n
        for p in self.peers.values():
            p.have = bytearray(n) if len(p.have) != n else p.have
        self._recount_wants()
        self.got_info.set()

    async def download_all(self) -> None:
        """Open storage, verify existing data (resume), start fetching all pieces."""
        assert self.info is not None
        os.makedirs(self.base_dir, exist_ok=True)
        # free-space preflight: what the layout still needs beyond the bytes on disk
        have = 0
        for p, n in self.info.file_paths(self.base_dir):
            if p:
                with contextlib.suppress(OSError):
                    have += min(os.path.getsize(p), n)
        check_space(self.base_dir, self.info.total_length - have, self.cfg.disk_reserve)
        self.db = CompletionDB(os.path.join(self.base_dir, ".torrent.db"))
        self.storage = FileStorage(self.base_dir, self.info, self.db)
        self.storage.open()
        if self.info.missing_layers():
            # pure v2 from a magnet: piece layers are not in the info dict;
            # fetch them (BEP 52 hash requests, merkle-proofed) before any piece
            # can be verified — resume check included
            await self._fetch_layers()
        loop = asyncio.get_running_loop()
        have = await loop.run_in_executor(None, self.storage.verify_existing, self.cfg.verify_device)
        for i in have:
            self.have[i] = 1
        self.nhave = len(have)
        self._recount_wants()
        self._init_file_tracking()
        if self.cfg.native_wire and _W is not None:
            n, pl, total = self.info.num_pieces, self.info.piece_length, self.info.total_length
            self.store = _W.PieceStore(n, pl, total)
            # the links answer block REQUESTs from the files themselves (own fd dups)
            src = _W.Source(n, pl, total)
            st = self.storage
            try:
                for fi, (_path, length) in enumerate(st.layout):
                    src.add_file(st.fd(fi), st.offsets[fi], length)
                src.set_have_bits(bytes(self.have))
                self.source = src
            except RuntimeError as e:            # e.g. out of descriptors: serve from Python instead
                src.close()
                log.with_field("error", str(e)).warn("native serving unavailable; requests answered in Python")
            for p in list(self.peers.values()):
                self._attach_link(p)
        self._downloading = True
        if self.nhave == self.info.num_pieces:
            self.complete.set()
        for p in list(self.peers.values()):
            self._send_have_state(p)
            self._update_interest(p)
            self._fill(p)

    # ------------------------------------------------------------ native data plane
    def _attach_link(self, p: _Peer) -> None:
        """Hand p's block traffic to a native link (csrc/btwire): from now on
        its peer loop feeds raw bytes to the link, which assembles blocks into
        the shared store and keeps requests pipelined over the pieces this
        Torrent assigns it."""
        if self.store is None or p.link is not None or p.wire.closed:
            return
        p.lid = next(self._lids)
        self._lid_key[p.lid] = p.key
        p.link = _W.Link(self.store, self.cfg.pipeline, p.hs.fast, p.lid)
        p.link.peer_choking = p.peer_choking
        if self.source is not None:
            p.link.set_source(self.source)

    def in_flight(self, i: int) -> bool:
        """Piece i is being fetched or verified (web seeds skip it)."""
        return i in self.pieces or i in self.verifying or (self.store is not None and self.store.active(i))

    def _unassign(self, p: _Peer, pieces=None) -> None:
        link = p.link
        if link is None:
            return
        for i in (link.assigned() if pieces is None else pieces):
            link.drop(i)
            s = self.assigned.get(i)
            if s is not None:
                s.discard(p.key)
                if not s:
                    del self.assigned[i]

    def _pick_piece(self, p: _Peer) -> int | None:
        """Next piece for p's link: a started piece nobody is fetching, else the
        rarest (watched-file order first) unstarted piece it has, else (end
        game) a piece other links are finishing."""
        assert self.store is not None
        have, store, assigned = self.have, self.store, self.assigned
        for i in store.active_pieces():
            if p.have[i] and not have[i] and not assigned.get(i) and i not in self.verifying and \
                    not self._isolated_from(i, p):
                return i
        order = self._rarest_order()
        pos = self._rare_pos
        while pos < len(order) and (have[order[pos]] or store.active(order[pos]) or order[pos] in self.verifying):
            pos += 1
        self._rare_pos = pos
        for k in range(pos, len(order)):
            i = order[k]
            if p.have[i] and not have[i] and not store.active(i) and i not in self.verifying \
                    and i not in self.ws_busy and not self._isolated_from(i, p):
                return i
        for i in store.active_pieces():
            owners = assigned.get(i, ())
            if p.have[i] and not have[i] and p.key not in owners and len(owners) < 3 and i not in self.verifying \
                    and not self._isolated_from(i, p):
                return i
        return None

    def _fill_native(self, p: _Peer) -> None:
        link = p.link
        if not p.peer_choking or p.hs.fast:
            while link.need_work():
                i = self._pick_piece(p)
                if i is None:
                    break
                link.assign(i)
                self.assigned.setdefault(i, set()).add(p.key)
        out = link.pump()
        if out:
            p.wire.send_raw(out)

    def _native_piece(self, src: _Peer, i: int) -> None:
        """A link completed piece i: take its bytes, stop the other links
        fetching it (end-game CANCELs), verify + write off-loop."""
        assert self.store is not None
        # who supplied which block (end game: several links), for blame on a hash failure
        keys = [self._lid_key.get(lid) if lid else None for lid in self.store.block_sources(i)]
        data = memoryview(self.store.take(i))     # pooled buffer, no copy
        for key in self.assigned.pop(i, set()):
            q = self.peers.get(key)
            if q is not None and q.link is not None:
                q.link.piece_done(i)
                if q is not src:
                    out = q.link.pump()
                    if out:
                        q.wire.send_raw(out)
        src.downloaded += len(data)
        self.downloaded += len(data)
        self.verifying.add(i)
        if self.info is not None and self.info.pieces:
            # v1 / hybrid: pieces are verified in groups, one executor hop per
            # group: 16 for the host's 16-lane AVX-512 SHA-1 (flushed after
            # VERIFY_WAIT_S if fewer arrive), else pairs in SHA-NI lockstep
            # (a lone piece goes at the end of this loop iteration)
            self._vq.append((i, data, keys))
            if len(self._vq) >= VERIFY_GROUP:
                self._submit_verify()
            elif not self._vflush:
                self._vflush = True
                loop = asyncio.get_running_loop()
                if VERIFY_GROUP > 2:
                    loop.call_later(VERIFY_WAIT_S, self._submit_verify)
                else:
                    loop.call_soon(self._submit_verify)
            return
        t = asyncio.get_running_loop().create_task(self._finish_native(i, data, keys))
        self._finishers.add(t)
        t.add_done_callback(self._finishers.discard)

    def _submit_verify(self) -> None:
        self._vflush = False
        if self.closed:                   # close() is draining: no writes may start now
            for i, _d, _s in self._vq:
                self.verifying.discard(i)
            self._vq.clear()
            return
        while self._vq:
            batch, self._vq = self._vq[:VERIFY_GROUP], self._vq[VERIFY_GROUP:]
            t = asyncio.get_running_loop().create_task(self._verify_batch(batch))
            self._finishers.add(t)
            t.add_done_callback(self._finishers.discard)

    async def _verify_batch(self, batch: list) -> None:
        assert self.info is not None and self.storage is not None
        info, st = self.info, self.storage

        def work() -> bytes:
            exp = b"".join(info.piece_hash(i) for i, _d, _s in batch)
            ok = hashing.verify_buffers("sha1", [d for _i, d, _s in batch], exp, 1)
            for (i, d, _s), good in zip(batch, ok):
                if good:
                    st.write(i, 0, d)
                    st.mark(i, True)
            return ok
        try:
            ok = await asyncio.get_running_loop().run_in_executor(None, work)
        except OSError as e:                  # the piece could not be written: the job cannot finish
            self._fatal(e)
            return
        finally:
            for i, _d, _s in batch:
                self.verifying.discard(i)
        for (i, d, keys), good in zip(batch, ok):
            if good:
                self._record_piece(i)
                self._good_piece(i, keys, d)
            else:
                self._bad_piece(i, keys, d)

    async def _finish_native(self, i: int, data: memoryview, keys: list) -> None:
        try:
            ok = await self.commit_piece(i, data)
        finally:
            self.verifying.discard(i)
        if ok is False:
            self._bad_piece(i, keys, data)
        elif ok:
            self._good_piece(i, keys, data)

    def _fatal(self, e: BaseException) -> None:
        """A storage error (disk full, I/O error): record it and wake whoever
        waits on ``failed`` — the job fails instead of waiting forever."""
        if self.fatal is None:
            self.fatal = e
            log.with_field("error", str(e)).error("torrent storage failed")
        self.failed.set()

    def _trust_of(self, key) -> list[int]:
        t = self.trust.get(key)
        if t is None:
            t = self.trust[key] = [0, 0]
        return t

    def _net(self, key) -> int:
        g, b = self.trust.get(key, (0, 0))
        return g - b

    def _good_piece(self, i: int, blocks, data=None) -> None:
        """Every peer that supplied blocks of a verified piece earns trust.  If
        the piece failed before, each block a peer sent then is compared with
        the verified data: a peer whose block differs sent corrupt data and is
        banned (smart ban: evidence, not a guess)."""
        self._isolate.pop(i, None)
        for k in dict.fromkeys(k for k in blocks if k is not None):
            self._trust_of(k)[0] += 1
            q = self.peers.get(k)
            if q is not None:
                q.good += 1
        sent = self._failed_blocks.pop(i, None)
        if sent and data is not None:
            mv = memoryview(data)
            for b, k, dg in sent:
                if k not in self.banned and _block_digest(mv, b) != dg:
                    log.with_fields(piece=i, block=b, peer=f"{k[0]}:{k[1]}").warn(
                        "peer sent a block that differs from the verified piece")
                    self._ban(k)

    def _bad_piece(self, i: int, blocks, data=None) -> None:
        """Piece i failed its hash (anacrolix ``pieceHashed`` with
        ``correct=false``, the default client of ``torrent.go:40-48``):
        ``blocks`` holds, per block, the key of the peer that supplied it.
        Every contributor is charged a bad piece, and the least trusted of
        them — fewest net good pieces — is banned at once; a piece one peer
        supplied alone bans that peer on its first failure.  When the least
        trusted are tied there is no evidence yet: nobody is banned, the
        blocks each peer sent are remembered (checked once the piece verifies,
        see :meth:`_good_piece`), and the piece is re-fetched from one of them
        only, so the next attempt either verifies (and convicts whoever sent
        a differing block) or fails with a single contributor.  An honest peer
        is therefore never banned, and a corrupter sharing every piece with it
        cannot stall the download."""
        keys = list(dict.fromkeys(k for k in blocks if k is not None))
        for k in keys:
            self._trust_of(k)[1] += 1
            q = self.peers.get(k)
            if q is not None:
                q.bad += 1
        log.with_fields(piece=i, peers=",".join(f"{k[0]}:{k[1]}" for k in keys)).warn("piece failed hash check")
        self._isolate.pop(i, None)
        victim = None
        if len(keys) == 1:
            victim = keys[0]
        elif keys:
            ranked = sorted(keys, key=self._net)
            if self._net(ranked[0]) < self._net(ranked[1]):
                victim = ranked[0]
        if len(keys) > 1 and data is not None:
            mv = memoryview(data)
            sent = self._failed_blocks.setdefault(i, [])
            for b, k in enumerate(blocks):
                if k is not None and len(sent) < 4096:
                    sent.append((b, k, _block_digest(mv, b)))
        if victim is not None:
            self._ban(victim)
        elif len(keys) > 1:
            # a tie: fetch it again from one contributor only — the most trusted, then
            # the one that supplied most of it
            pick = max(keys, key=lambda k: (self._net(k), sum(1 for x in blocks if x == k)))
            self._isolate[i] = pick
        self._rare_dirty = True
        for q in list(self.peers.values()):
            if q.link is not None:
                self._fill(q)

    def _isolated_from(self, i: int, p: _Peer) -> bool:
        """Piece i is being re-fetched from another single peer (still connected)."""
        k = self._isolate.get(i)
        return k is not None and k != p.key and k in self.peers

    async def _native_loop(self, p: _Peer) -> None:
        data = await p.wire.read_raw()
        p.last_recv = time.monotonic()
        await self._native_feed(p, data)

    async def _native_feed(self, p: _Peer, data: bytes) -> None:
        while True:
            msgs: list = []
            self._native_events(p, *p.link.feed(data), msgs.append)
            for m in msgs:
                await self._dispatch(p, m[0], m[1])
            if not p.link.stalled or p.wire.closed or self.closed:
                return
            await p.wire.drain()      # served up to the budget: let it drain, then parse the rest
            data = b""

    def _native_recv(self, p: _Peer, nbytes: int) -> None:
        """LinkReader callback: nbytes landed in p.link's buffer (zero-copy)."""
        p.last_recv = time.monotonic()
        self._native_events(p, *p.link.feed_n(nbytes), lambda m: p.rx.push(m[0], m[1]))

    def _native_recv_bytes(self, p: _Peer, data: bytes) -> None:
        """UtpLinkReader callback: bytes the uTP engine delivered for p."""
        p.last_recv = time.monotonic()
        self._native_events(p, *p.link.feed(data), lambda m: p.rx.push(m[0], m[1]))

    def _native_events(self, p: _Peer, ev, out: bytes, defer) -> None:
        """Act on what a link parsed: pieces and choke state here and now;
        other messages go to ``defer`` for the (async) dispatcher."""
        if out:
            p.wire.send_raw(out)
        for e in ev:
            kind = e[0]
            if kind == "msg":
                defer((e[1], e[2]))
            elif kind == "piece":
                self._native_piece(p, e[1])
            elif kind == "unchoke":
                p.peer_choking = False
            elif kind == "choke":
                p.peer_choking = True
                if not p.hs.fast:
                    self._unassign(p)          # its pieces go back to the other links
                    for q in list(self.peers.values()):
                        if q is not p and q.link is not None:
                            self._fill(q)
            elif kind == "bad":
                raise pw.PeerError(e[1])
        if not self.closed and self.info is not None:
            self._fill(p)

    # ------------------------------------------------------------ per-file completion
    def watch_files(self, pick, on_complete) -> None:
        """Stream files out as they finish instead of after the whole torrent.

        ``pick(paths)`` is called once storage is laid out with every file's
        path and returns the subset to watch; ``on_complete(path)`` fires (on
        the loop) when the last piece covering a watched file is verified and
        written — at once for files the resume check already found whole.
        Watched files also move to the front of the piece picker, in layout
        order (rarest-first within each file), so they finish one by one.
        The reference uploaded only after ``WaitAll`` (``torrent.go:104-113``
        → ``downloader.go:122-133``); this lets the uploads overlap the swarm.
        Must be called before :meth:`download_all`."""
        self._file_pick, self._file_cb = pick, on_complete

    def _init_file_tracking(self) -> None:
        if self._file_cb is None or self.info is None or self.storage is None:
            return
        layout = self.storage.layout
        picked = self._file_pick([p for p, _n in layout if p]) if self._file_pick else set()
        pl = self.info.piece_length
        n = self.info.num_pieces
        rank = [len(layout)] * n
        done: list[str] = []
        for fi, (path, length) in enumerate(layout):
            if not path or path not in picked:
                continue
            off = self.info.files[fi].offset
            if length == 0:
                done.append(path)
                continue
            first, last = off // pl, (off + length - 1) // pl
            left = 0
            for i in range(first, last + 1):
                rank[i] = min(rank[i], fi)
                if not self.have[i]:
                    left += 1
                    self._piece_files.setdefault(i, []).append(fi)
            if left:
                self._file_left[fi] = left
            else:
                done.append(path)
        if picked:
            self._piece_rank = rank
            self._rare = None
        for path in done:
            self._file_cb(path)

    def _note_piece(self, i: int) -> None:
        fis = self._piece_files.pop(i, None)
        if not fis:
            return
        assert self.storage is not None
        for fi in fis:
            left = self._file_left[fi] - 1
            if left:
                self._file_left[fi] = left
            else:
                del self._file_left[fi]
                self._file_cb(self.storage.layout[fi][0])

    def bytes_completed(self) -> int:
        if self.info is None:
            return 0
        done = sum(self.info.piece_size(i) for i in range(self.info.num_pieces) if self.have[i])
        partial = sum(len(pc.received) * BLOCK for pc in self.pieces.values())
        if self.store is not None:
            partial += self.store.partial_bytes
        return min(done + partial, self.info.total_length)

    # ------------------------------------------------------------ discovery
    def add_peer_addrs(self, addrs) -> None:
        """A batch from a tracker / the DHT: all become known, and the free
        connection slots go to the highest BEP 40 priority ones."""
        for a in addrs:
            if not self.closed and a not in self.banned and a[1] > 0 and \
                    not (a[1] == self.port and a[0] in ("127.0.0.1", "0.0.0.0", self.cfg.announce_host)):
                self._remember(a)
        free = self._dial_slots()
        if free > 0:
            for a in self._best_candidates(free):
                self.add_peer_addr(a)

    def add_peer_addr(self, addr: tuple[str, int]) -> None:
        if self.closed or addr in self.banned or addr[1] <= 0:
            return
        if addr in self.peers or addr in self.connecting:
            return
        if addr[1] == self.port and addr[0] in ("127.0.0.1", "0.0.0.0", self.cfg.announce_host):
            return
        self._remember(addr)
        if self._dial_slots() > 0:
            self.connecting.add(addr)
            self._spawn(self._connect(addr))

    def _remember(self, a: tuple[str, int]) -> None:
        """Add ``a`` to the known addresses, bounded at ``peers_high_water``:
        a PEX or tracker flood cannot grow the set without limit."""
        if a in self.known:
            return
        if len(self.known) >= self.cfg.peers_high_water:
            for old in self.known:
                if old not in self.peers and old not in self.connecting:
                    self.known.discard(old)      # the loop ends here: no further iteration
                    break
            else:
                return                           # every known address is in use
        self.known.add(a)

    def _dial_slots(self) -> int:
        """Dials that may start now: half-open connections are capped at
        ``half_open_conns`` and established + half-open at ``established_conns``
        (anacrolix ``HalfOpenConnsPerTorrent`` / ``EstablishedConnsPerTorrent``)."""
        return min(self.cfg.half_open_conns - len(self.connecting),
                   self.cfg.established_conns - len(self.peers) - len(self.connecting))

    async def _tracker_loop(self, url: str) -> None:
        event = "started"
        while not self.closed:
            left = (self.info.total_length - self.bytes_completed()) if self.info else 1 << 40
            a = Announce(self.infohash, self.peer_id, self.port, self.uploaded, self.downloaded, left, event)
            interval = self.cfg.tracker_min_interval
            try:
                res = await announce(url, a)
                self.add_peer_addrs(res.peers)
                interval = max(self.cfg.tracker_min_interval, min(res.interval, 1800))
                event = ""
            except (TrackerError, OSError) as e:
                log.with_fields(tracker=url, error=str(e)).debug("tracker announce failed")
            if self.complete.is_set() and event != "completed" and event == "":
                with contextlib.suppress(TrackerError, OSError):
                    await announce(url, Announce(self.infohash, self.peer_id, self.port, self.uploaded,
                                                 self.downloaded, 0, "completed"))
                event = "done"
            await asyncio.sleep(interval if not self._starving() else min(interval, 5.0))

    def _accepts(self, ih: bytes) -> bool:
        """Our 20-byte info-hash, or (hybrid) the truncated v2 one."""
        return ih == self.infohash or (self.info is not None and bool(self.info.infohash_v2)
                                       and ih == self.info.infohash_v2[:20])

    @property
    def private(self) -> bool:
        return bool(self.info is not None and self.info.private)

    def _starving(self) -> bool:
        return not self.peers

    async def _dht_loop(self) -> None:
        assert self.dht is not None
        while not self.closed:
            if self.private:
                return                   # BEP 27: private torrents use their trackers only
            try:
                self.add_peer_addrs(await self.dht.get_peers(self.infohash))
                await self.dht.announce_peer(self.infohash, self.port)
            except Exception as e:  # noqa: BLE001 - discovery is best-effort
                log.with_field("error", str(e)).debug("dht lookup failed")
            await asyncio.sleep(self.cfg.dht_interval if self.peers else min(self.cfg.dht_interval, 5.0))

    # ------------------------------------------------------------ connections
    async def _dial_tcp(self, addr: tuple[str, int]):
        # fast fallback for a peer given by name (BEP 3 dictionary peer lists; anacrolix
        # dials through Go's net.Dialer); an IP literal is one address, dialled directly
        return await tcpdial.open_connection(addr[0], addr[1], timeout=self.cfg.connect_timeout)

    async def _dial_utp(self, addr: tuple[str, int]):
        assert self.utp is not None
        return await self.utp.connect(addr[0], addr[1], self.cfg.connect_timeout)

    async def _dial_and_handshake(self, dial, addr):
        policy = self.cfg.encryption
        ours = pw.encode_handshake(self.infohash, self.peer_id)
        if policy in ("prefer", "require"):
            reader, writer = await dial(addr)
            try:
                provide = mse.CRYPTO_RC4 if policy == "require" else mse.CRYPTO_RC4 | mse.CRYPTO_PLAIN
                reader, writer, _sel = await mse.initiate(reader, writer, self.infohash, ours, provide,
                                                          self.cfg.connect_timeout)
                hs = await asyncio.wait_for(pw.read_handshake(reader), self.cfg.connect_timeout)
                return reader, writer, hs
            except BaseException as e:
                writer.close()
                if policy == "require" or not isinstance(e, (OSError, asyncio.TimeoutError,
                                                             asyncio.IncompleteReadError, pw.PeerError)):
                    raise
                # "prefer": the peer does not speak MSE; redial in plaintext
        reader, writer = await dial(addr)
        try:
            writer.write(ours)
            hs = await asyncio.wait_for(pw.read_handshake(reader), self.cfg.connect_timeout)
        except BaseException:
            writer.close()
            raise
        return reader, writer, hs

    async def _connect(self, addr: tuple[str, int]) -> None:
        """Dial TCP and (if enabled) uTP concurrently; the first transport to
        complete the BitTorrent handshake wins (anacrolix dials both too)."""
        dials = [self._dial_tcp] + ([self._dial_utp] if self.utp is not None else [])
        tasks = [asyncio.ensure_future(self._dial_and_handshake(d, addr)) for d in dials]
        won = None
        try:
            for fut in asyncio.as_completed(tasks):
                try:
                    won = await fut
                    break
                except (OSError, asyncio.TimeoutError, asyncio.IncompleteReadError, pw.PeerError, ConnectionError):
                    continue
        finally:
            for t in tasks:
                if not t.done():
                    t.cancel()
            for t in tasks:
                if t.done() and not t.cancelled() and t.exception() is None and t.result() is not won:
                    t.result()[1].close()
        self.connecting.discard(addr)
        if won is None:
            return
        reader, writer, hs = won
        await self._run_peer(reader, writer, addr, hs, inbound=False)

    async def _on_inbound(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        addr = writer.get_extra_info("peername")[:2]
        sock = writer.get_extra_info("socket")
        if sock is not None:
            with contextlib.suppress(OSError):
                tcpdial.tcp_options(sock)      # Go's net.ListenConfig: keep-alive on accepted conns too
        policy = self.cfg.encryption
        try:
            first = await asyncio.wait_for(reader.readexactly(len(mse.PLAIN_PREFIX)), self.cfg.connect_timeout)
            if first == mse.PLAIN_PREFIX:
                if policy == "require":
                    raise pw.PeerError("plaintext connection refused (encryption required)")
                rest = await asyncio.wait_for(reader.readexactly(pw.HANDSHAKE_LEN - len(first)),
                                              self.cfg.connect_timeout)
                hs = pw.parse_handshake(first + rest)
            else:
                if policy == "disable":
                    raise pw.PeerError("encrypted connection refused (encryption disabled)")
                reader, writer, _sel = await mse.respond(reader, writer, first, self.infohash,
                                                         allow_plain=policy != "require",
                                                         timeout=self.cfg.connect_timeout)
                hs = await asyncio.wait_for(pw.read_handshake(reader), self.cfg.connect_timeout)
            if not self._accepts(hs.infohash):
                writer.close()
                return
            writer.write(pw.encode_handshake(hs.infohash, self.peer_id))   # answer with the hash they used
        except (OSError, asyncio.TimeoutError, asyncio.IncompleteReadError, pw.PeerError):
            writer.close()
            return
        await self._run_peer(reader, writer, addr, hs, inbound=True)

    async def _run_peer(self, reader, writer, addr, hs: pw.Handshake, inbound: bool = True) -> None:
        if not self._accepts(hs.infohash) or hs.peer_id == self.peer_id or addr in self.peers or self.closed or \
                (inbound and len(self.peers) >= self.cfg.established_conns):
            writer.close()
            return
        n = self.info.num_pieces if self.info else 0
        if self._my_ip is None:           # our address as peers see it (BEP 40 priorities)
            sn = writer.get_extra_info("sockname")
            self._my_ip = self.cfg.announce_host or (sn[0] if sn else None)
        p = _Peer(pw.Wire(reader, writer), addr, hs, n)
        if not inbound:
            p.listen_addr = addr
        self.peers[addr] = p
        self._attach_link(p)
        try:
            if hs.extended:
                p.wire.ext_handshake(len(self.info.raw) if self.info else None, self.port,
                                     pex=self.cfg.pex and not self.private)
            if self.info is not None and self._downloading:
                self._send_have_state(p)
            await self._peer_loop(p)
        except (OSError, asyncio.IncompleteReadError, pw.PeerError, ConnectionError, struct.error) as e:
            # struct.error: a message shorter than its type's fixed fields (protocol violation)
            log.with_fields(peer=f"{addr[0]}:{addr[1]}", error=str(e) or type(e).__name__).debug("peer closed")
        finally:
            self._drop_peer(p)

    @property
    def uploaded(self) -> int:
        """Bytes served to peers (tracker ``uploaded``), native links included."""
        return self._uploaded + sum(p.link.uploaded for p in self.peers.values() if p.link is not None)

    def _drop_peer(self, p: _Peer) -> None:
        p.wire.close()
        if self.peers.get(p.key) is p:
            del self.peers[p.key]
            if p.link is not None:
                self._uploaded += p.link.uploaded
        if self.info is not None:
            for i in range(len(p.have)):
                if p.have[i] and i < len(self.avail):
                    self.avail[i] -= 1
                    self._rare_dirty = True
        self._release(p)
        # top up from known addresses, highest BEP 40 priority first (as anacrolix dials)
        for a in self._best_candidates(4):
            self.add_peer_addr(a)

    def _best_candidates(self, k: int) -> list[tuple[str, int]]:
        cands = self.known - set(self.peers) - self.connecting - self.banned
        if not cands:
            return []
        mine = (self._my_ip or self.cfg.announce_host or "0.0.0.0", self.port)
        prio = self._prio

        def key(a: tuple[str, int]) -> int:
            v = prio.get(a)
            if v is None:
                v = prio[a] = bep40.priority(mine, a)
            return v
        return heapq.nlargest(k, cands, key=key)

    def _release(self, p: _Peer) -> None:
        if p.link is not None:
            self._unassign(p)
            for q in list(self.peers.values()):
                if q is not p:
                    self._fill(q)
            return
        for (i, off) in list(p.outstanding):
            pc = self.pieces.get(i)
            if pc is not None and pc.lapse(off // BLOCK, p.key):
                self.open_pieces[i] = pc
        p.outstanding.clear()
        for q in self.peers.values():
            if q is not p:
                self._fill(q)

    def _send_have_state(self, p: _Peer) -> None:
        assert self.info is not None
        n = self.info.num_pieces
        if p.hs.fast and self.nhave == n:
            p.wire.send(pw.HAVE_ALL)
        elif p.hs.fast and self.nhave == 0:
            p.wire.send(pw.HAVE_NONE)
        elif self.nhave:
            p.wire.bitfield(pw.set_to_bits(list(map(bool, self.have)), n))
        p.wire.send(pw.UNCHOKE)  # we unchoke everyone (no tit-for-tat needed for a leech/seed job)

    # ------------------------------------------------------------ peer loop
    async def _peer_loop(self, p: _Peer) -> None:
        last_drain = time.monotonic()
        p.last_recv = time.monotonic()
        while not self.closed:
            if p.link is not None:
                if p.rx is None and not p.rx_tried:
                    p.rx_tried = True
                    r = p.wire.take_over(p.link, functools.partial(self._native_recv, p),
                                         functools.partial(self._native_recv_bytes, p))
                    if r is not None:
                        p.rx, leftover = r
                        if leftover:
                            await self._native_feed(p, leftover)
                if p.rx is not None:
                    for m in await p.rx.get():
                        await self._dispatch(p, m[0], m[1])
                else:
                    await self._native_loop(p)
            else:
                msgs = await p.wire.read_batch()
                p.last_recv = time.monotonic()
                if p.link is not None:
                    # the native link took over while this read was pending: these
                    # messages (block replies to its requests included) are its input
                    await self._native_feed(p, b"".join(
                        struct.pack(">IB", len(m[1]) + 1, m[0]) + m[1] if m is not None else b"\0\0\0\0"
                        for m in msgs))
                    continue
                for m in msgs:
                    if m is None:
                        continue
                    await self._dispatch(p, m[0], m[1])
            now = time.monotonic()
            if now - last_drain > 0.5 or p.wire.writer.transport.get_write_buffer_size() > (4 << 20):
                last_drain = now
                await p.wire.drain()

    async def _dispatch(self, p: _Peer, mid: int, pl: bytes) -> None:
        if mid == pw.PIECE:
            await self._on_block(p, pl)
        elif mid == pw.HAVE:
            (i,) = struct.unpack(">I", pl[:4])
            self._peer_has(p, [i])
        elif mid == pw.BITFIELD:
            if self.info is not None:
                self._peer_has(p, sorted(pw.bits_to_set(pl, self.info.num_pieces)))
            else:
                p.pending_bitfield = pl  # type: ignore[attr-defined]
        elif mid == pw.HAVE_ALL:
            if self.info is not None:
                self._peer_has(p, range(self.info.num_pieces))
            else:
                p.pending_have_all = True  # type: ignore[attr-defined]
        elif mid == pw.HAVE_NONE:
            pass
        elif mid == pw.UNCHOKE:
            p.peer_choking = False
            if p.link is not None:          # parsed by Python just before the native link took over
                p.link.peer_choking = False
            self._fill(p)
        elif mid == pw.CHOKE:
            p.peer_choking = True
            if p.link is not None:
                p.link.peer_choking = True
            if not p.hs.fast:
                self._release(p)
        elif mid == pw.INTERESTED:
            p.peer_interested = True
        elif mid == pw.NOT_INTERESTED:
            p.peer_interested = False
        elif mid == pw.REQUEST:
            self._on_request(p, pl)
        elif mid == pw.REJECT:
            i, off, _n = struct.unpack(">III", pl[:12])
            self._unrequest(p, i, off)
            self._fill(p)
        elif mid == pw.CANCEL:
            pass
        elif mid == pw.EXTENDED:
            await self._on_extended(p, pl)
        elif mid in (pw.HASH_REQUEST, pw.HASHES, pw.HASH_REJECT):
            self._on_hash_msg(p, mid, pl)

    def _peer_has(self, p: _Peer, idxs) -> None:
        if self.info is None:
            return
        have = self.have
        for i in idxs:
            if p.set_have(i):
                self.avail[i] += 1
                self._rare_dirty = True
                if not have[i]:
                    p.wants += 1
        self._update_interest(p)
        self._fill(p)

    def _wants(self, p: _Peer) -> bool:
        """Does p have any piece we lack?  O(1): p.wants counts them, kept by
        _peer_has / _record_piece and recounted when our bitmap jumps (resume)."""
        return p.wants > 0

    def _recount_wants(self) -> None:
        mine = ~int.from_bytes(self.have, "little")
        for p in self.peers.values():
            p.wants = (int.from_bytes(p.have, "little") & mine).bit_count() if len(p.have) == len(self.have) else 0

    def _update_interest(self, p: _Peer) -> None:
        if self.info is None or not self._downloading:
            return
        want = self._wants(p) if p.nhave else False
        if want != p.am_interested:
            p.am_interested = want
            p.wire.send(pw.INTERESTED if want else pw.NOT_INTERESTED)

    # ------------------------------------------------------------ requests
    def _rarest_order(self) -> list[int]:
        now = time.monotonic()
        if self._rare is None or (self._rare_dirty and now - self._rare_t > 0.25) or \
                self._rare_pos >= len(self._rare):
            idx = [i for i in range(len(self.have)) if not self.have[i]]
            random.shuffle(idx)
            rank = self._piece_rank
            if rank is None:
                idx.sort(key=self.avail.__getitem__)
            else:                          # watched files first, in order; rarest-first within
                av = self.avail
                idx.sort(key=lambda i: (rank[i], av[i]))
            self._rare, self._rare_t, self._rare_dirty, self._rare_pos = idx, now, False, 0
        return self._rare

    def _pick(self, p: _Peer) -> tuple[int, int, int] | None:
        """Next (piece, offset, length) to request from p; None if nothing."""
        assert self.info is not None
        # 1) continue in-progress pieces that still have unrequested blocks
        exhausted = []
        try:
            for i, pc in self.open_pieces.items():
                if not p.have[i] or self._isolated_from(i, p):
                    continue
                b = pc.take()
                if b is not None:
                    return i, b * BLOCK, min(BLOCK, pc.size - b * BLOCK)
                exhausted.append(i)
        finally:
            for i in exhausted:
                del self.open_pieces[i]
        # 2) start the rarest piece this peer has (random tie-break), from an
        #    availability-ordered list refreshed at most every 0.25 s — a full
        #    scan per new piece was O(pieces^2) over a download
        best = None
        order = self._rarest_order()
        pos = self._rare_pos
        while pos < len(order) and (self.have[order[pos]] or order[pos] in self.pieces
                                    or order[pos] in self.verifying):
            pos += 1                       # taken for good (until the next refresh)
        self._rare_pos = pos
        for k in range(pos, len(order)):
            i = order[k]
            if p.have[i] and not self.have[i] and i not in self.pieces and i not in self.verifying \
                    and i not in self.ws_busy and not self._isolated_from(i, p):
                best = i
                break
        if best is not None:
            size = self.info.piece_size(best)
            pc = _Piece(size, -(-size // BLOCK), bytearray(size))
            self.pieces[best] = pc
            pc.next_b = 1
            if pc.nblocks > 1:
                self.open_pieces[best] = pc
            return best, 0, min(BLOCK, size)
        # 3) end game: duplicate outstanding requests of other peers
        for i, pc in self.pieces.items():
            if not p.have[i] or self._isolated_from(i, p):
                continue
            for b, who in pc.requested.items():
                if b not in pc.received and p.key not in who and len(who) < 3:
                    return i, b * BLOCK, min(BLOCK, pc.size - b * BLOCK)
        return None

    def _fill(self, p: _Peer) -> None:
        if p.link is not None:
            if self.info is not None and self._downloading and not p.wire.closed and not self.complete.is_set():
                self._fill_native(p)
            return
        if self.info is None or not self._downloading or p.peer_choking or p.wire.closed:
            return
        while len(p.outstanding) < self.cfg.pipeline:
            nxt = self._pick(p)
            if nxt is None:
                break
            i, off, n = nxt
            pc = self.pieces[i]
            pc.requested.setdefault(off // BLOCK, set()).add(p.key)
            p.outstanding[(i, off)] = time.monotonic()
            p.wire.request(i, off, n)

    def _unrequest(self, p: _Peer, i: int, off: int) -> None:
        if p.outstanding.pop((i, off), None) is not None:
            p.withdrew((i, off))
        pc = self.pieces.get(i)
        if pc is not None and pc.lapse(off // BLOCK, p.key):
            self.open_pieces[i] = pc

    async def _on_block(self, p: _Peer, pl: bytes) -> None:
        i, off = struct.unpack(">II", pl[:8])
        data = pl[8:]
        if p.outstanding.pop((i, off), None) is None and not p.recent.pop((i, off), 0):
            # never asked of this peer (nor recently withdrawn): a peer pushing blocks
            # could poison pieces other peers are filling, so the bytes are dropped
            p.wasted += len(data)
            self.wasted += len(data)
            self._fill(p)
            return
        pc = self.pieces.get(i)
        if pc is None or self.info is None or self.have[i]:
            self._fill(p)
            return
        b = off // BLOCK
        if off % BLOCK or b >= pc.nblocks or off + len(data) > pc.size:
            raise pw.PeerError("bad block geometry")
        if b not in pc.received:
            pc.buf[off:off + len(data)] = data
            pc.received.add(b)
            pc.src[b] = p.key
            p.downloaded += len(data)
            self.downloaded += len(data)
            # cancel duplicates (end game)
            for other in pc.requested.pop(b, set()):
                q = self.peers.get(other)
                if q is not None and q is not p and (i, off) in q.outstanding:
                    q.outstanding.pop((i, off), None)
                    q.withdrew((i, off))
                    q.wire.cancel(i, off, len(data))
        else:
            pc.requested.pop(b, None)
        if len(pc.received) == pc.nblocks:
            # hash+write off-loop; keep requesting meanwhile (the piece stays
            # out of the picker via `verifying` until it lands or fails)
            del self.pieces[i]
            self.open_pieces.pop(i, None)
            self.verifying.add(i)
            t = asyncio.get_running_loop().create_task(self._finish_piece(i, pc, p))
            self._finishers.add(t)
            t.add_done_callback(self._finishers.discard)
        self._fill(p)

    async def _finish_piece(self, i: int, pc: _Piece, src: _Peer) -> None:
        blocks = [pc.src.get(b, src.key) for b in range(pc.nblocks)]
        ok = await self.commit_piece(i, pc.buf)   # the buffer is no longer shared: the piece left self.pieces
        if ok is None:
            return                                # unverifiable yet (v2 layer missing): not the peer's fault
        if ok:
            self._good_piece(i, blocks, pc.buf)
        else:
            self._bad_piece(i, blocks, pc.buf)
            for q in list(self.peers.values()):
                if q.link is None and not q.wire.closed:
                    self._fill(q)

    def _ban(self, key) -> None:
        """No more connections to (or from) this peer address; drop it now."""
        self.banned.add(key)
        q = self.peers.get(key)
        log.with_fields(peer=f"{key[0]}:{key[1]}", trust=self._net(key)).warn("banning peer for bad pieces")
        if q is not None:
            q.wire.close()

    async def commit_piece(self, i: int, data) -> bool | None:
        """Verify a whole piece off-loop, write it and record completion; then
        announce it.  Shared by peer downloads and web seeds.  False on a hash
        mismatch (nothing is written)."""
        assert self.info is not None and self.storage is not None
        loop = asyncio.get_running_loop()
        st = self.storage

        info = self.info

        def verify_and_write() -> bool | None:
            ok = info.check_piece(i, data)
            if not ok:
                return ok                    # False: bad data; None: v2 piece layer unknown
            st.write(i, 0, data)
            st.mark(i, True)
            return True

        self.verifying.add(i)
        try:
            ok = await loop.run_in_executor(None, verify_and_write)
        except OSError as e:
            self._fatal(e)
            return None
        finally:
            self.verifying.discard(i)
        if not ok:
            return ok
        self._record_piece(i)
        return True

    def _record_piece(self, i: int) -> None:
        """Piece i is verified and written: mark it, announce it, update
        interest, per-file completion and the torrent's completion."""
        assert self.info is not None
        if self.have[i]:
            return
        self.have[i] = 1
        self.nhave += 1
        if self.source is not None:
            self.source.set_have(i)
        for q in list(self.peers.values()):
            q.wire.have(i)
            if q.have[i]:
                q.wants -= 1
            if q.am_interested and q.have[i] and not self._wants(q):
                q.am_interested = False
                q.wire.send(pw.NOT_INTERESTED)
        if self._piece_files:
            self._note_piece(i)
        if self.nhave == self.info.num_pieces:
            self.complete.set()

    def _on_request(self, p: _Peer, pl: bytes) -> None:
        i, off, n = struct.unpack(">III", pl[:12])
        if self.info is None or self.storage is None or i >= len(self.have) or not self.have[i] or \
                n > 128 * 1024 or off + n > self.info.piece_size(i):
            if p.hs.fast:
                p.wire.reject(i, off, n)
            return
        # a 16 KiB pread from the page cache costs less than a thread hop
        data = self.storage.read(i, off, n)
        p.wire.piece(i, off, data)
        self._uploaded += len(data)

    async def _timeout_loop(self) -> None:
        while not self.closed:
            await asyncio.sleep(2.0)
            now = time.monotonic()
            for p in list(self.peers.values()):
                if now - getattr(p, "last_keepalive", 0) > 90:
                    p.last_keepalive = now  # type: ignore[attr-defined]
                    p.wire.keepalive()
                if now - getattr(p, "last_recv", now) > 300:
                    p.wire.close()  # silent for 5 minutes: drop
                    continue
                if p.link is not None:
                    if p.link.outstanding and p.link.oldest_request_age() > self.cfg.request_timeout:
                        p.link.lapse_all()
                        self._unassign(p)
                        p.peer_choking = p.link.peer_choking = True   # snubbed until it sends something
                        for q in list(self.peers.values()):
                            if q is not p:
                                self._fill(q)
                    continue
                stale = [k for k, t in p.outstanding.items() if now - t > self.cfg.request_timeout]
                if stale and len(stale) == len(p.outstanding):
                    for (i, off) in stale:
                        self._unrequest(p, i, off)
                    p.peer_choking = True  # treat as snubbed until it sends something
                    for q in self.peers.values():
                        if q is not p:
                            self._fill(q)
            # metadata retry
            if self.info is None:
                for p in self.peers.values():
                    if p.ext and "ut_metadata" in p.ext.m and self._meta_size:
                        self._request_metadata(p)

    async def _pex_loop(self) -> None:
        """BEP 11: every ``pex_interval`` tell each ut_pex-capable peer which
        dialable peers joined / left since the last message to it."""
        while not self.closed:
            await asyncio.sleep(self.cfg.pex_interval)
            if self.private:
                return
            self.pex_round()

    def pex_round(self) -> None:
        live = {q.listen_addr: q for q in self.peers.values() if q.listen_addr is not None}
        for p in list(self.peers.values()):
            their = p.ext.m.get("ut_pex") if p.ext else None
            if not their or p.wire.closed:
                continue
            cur = set(live) - {p.listen_addr}
            added = [a for a in cur if a not in p.pex_sent][:pw.PEX_MAX_ADDED]
            dropped = [a for a in p.pex_sent if a not in cur][:pw.PEX_MAX_ADDED]
            if not added and not dropped:
                continue
            flags = {}
            for a in added:
                q = live[a]
                f = 0x10                                   # we dialled / it told us its port
                if q.nhave and q.nhave == len(q.have):
                    f |= 0x02
                if type(q.wire.writer.transport).__name__ == "_UtpTransport":
                    f |= 0x04                              # reached over uTP
                flags[a] = f
            p.wire.extended(their, pw.pex_msg(added, dropped, flags))
            p.pex_sent.update(added)
            p.pex_sent.difference_update(dropped)

    # ------------------------------------------------------------ BEP 52 piece layers
    def _layer_geometry(self, f) -> tuple[int, int, int]:
        """(base layer, request length, proof layers) for fetching f's piece layer."""
        assert self.info is not None
        base = merkle.piece_levels(self.info.piece_length)
        width = merkle.next_pow2(f.num_pieces)
        length = min(512, width)
        total_h = width.bit_length() - 1
        return base, length, total_h - (length.bit_length() - 1)

    def _on_hash_msg(self, p: _Peer, mid: int, pl: bytes) -> None:
        root, base, index, length, proofs, hashes = pw.parse_hash_msg(pl)
        info = self.info
        if mid == pw.HASH_REQUEST:
            layer = info.piece_layers.get(root) if info is not None else None
            ans = None
            if layer is not None and base == merkle.piece_levels(info.piece_length) and length <= 512:
                nodes = [layer[k:k + 32] for k in range(0, len(layer), 32)]
                ans = merkle.serve_hashes(nodes, base, index, length, proofs)
            if ans is None:
                p.wire.hash_reject(root, base, index, length, proofs)
            else:
                p.wire.hashes(root, base, index, length, proofs, ans)
            return
        fut = self._layer_waiters.pop((root, index, p.key), None)
        if fut is None or fut.done():
            return
        if mid == pw.HASH_REJECT or info is None:
            fut.set_result(None)
            return
        f = next((x for x in info.v2_files if x.root == root), None)
        got = merkle.check_hashes(root, base, index, length, hashes, f.num_pieces) if f is not None else None
        fut.set_result(got)

    async def _fetch_layers(self, timeout: float | None = None) -> None:
        """Fetch every missing piece layer in merkle-proofed slices of <= 512
        hashes from v2-capable peers, trying peers in turn per slice."""
        assert self.info is not None
        info = self.info
        deadline = time.monotonic() + (timeout if timeout is not None else self.cfg.layer_timeout)
        for f in info.missing_layers():
            base, length, proofs = self._layer_geometry(f)
            slices: dict[int, list[bytes]] = {}
            for index in range(0, f.num_pieces, length):
                tried: set = set()
                while index not in slices:
                    if time.monotonic() > deadline or self.closed:
                        raise MetainfoError(f"could not fetch the piece layer of {'/'.join(f.path)}")
                    cands = [q for q in self.peers.values() if q.hs.v2 and q.key not in tried and not q.wire.closed]
                    if not cands:
                        tried.clear()
                        await asyncio.sleep(0.2)
                        continue
                    q = cands[0]
                    tried.add(q.key)
                    fut = asyncio.get_running_loop().create_future()
                    self._layer_waiters[(f.root, index, q.key)] = fut
                    q.wire.hash_request(f.root, base, index, length, proofs)
                    try:
                        got = await asyncio.wait_for(fut, 10.0)
                    except asyncio.TimeoutError:
                        got = None
                    finally:
                        self._layer_waiters.pop((f.root, index, q.key), None)
                    if got is not None:
                        slices[index] = got
            layer = b"".join(h for k in sorted(slices) for h in slices[k])[:32 * f.num_pieces]
            if not info.set_piece_layer(f.root, layer):
                raise MetainfoError("fetched piece layer does not reduce to its pieces root")
        log.with_field("files", len(info.v2_files)).debug("v2 piece layers complete")

    # ------------------------------------------------------------ extensions
    async def _on_extended(self, p: _Peer, pl: bytes) -> None:
        if not pl:
            return
        eid, body = pl[0], pl[1:]
        if eid == pw.EXT_HANDSHAKE:
            p.ext = pw.parse_ext_handshake(body)
            if p.listen_addr is None and p.ext.port and 0 < p.ext.port < 65536:
                p.listen_addr = (p.addr[0], p.ext.port)
            if self.info is None and "ut_metadata" in p.ext.m and p.ext.metadata_size:
                if self._meta_size is None and p.key not in self._meta_bad and \
                        0 < p.ext.metadata_size < 16 * 1024 * 1024:
                    self._meta_size = p.ext.metadata_size
                self._request_metadata(p)
            return
        if eid == pw.UT_PEX_ID:
            if not self.cfg.pex or self.private:
                return
            added, _dropped = pw.parse_pex(body)
            for a in added[:pw.PEX_MAX_ADDED]:
                if a not in self.known and a not in self.peers:
                    self.pex_learned += 1
                self.add_peer_addr(a)
            return
        if eid == pw.UT_METADATA_ID:
            d, data = pw.parse_meta_msg(body)
            t, piece = d.get(b"msg_type"), d.get(b"piece")
            if t == pw.META_REQUEST:
                their = (p.ext.m.get("ut_metadata") if p.ext else None)
                if not their:
                    return
                if self.info is None or not isinstance(piece, int) or not 0 <= piece * BLOCK < len(self.info.raw):
                    p.wire.extended(their, pw.meta_msg(pw.META_REJECT, piece if isinstance(piece, int) else 0))
                else:
                    raw = self.info.raw
                    p.wire.extended(their, pw.meta_msg(pw.META_DATA, piece, len(raw),
                                                       raw[piece * BLOCK:(piece + 1) * BLOCK]))
            elif t == pw.META_DATA and self.info is None and isinstance(piece, int) and self._meta_size \
                    and 0 <= piece < -(-self._meta_size // BLOCK) and len(data) <= BLOCK \
                    and p.key not in self._meta_bad and d.get(b"total_size", self._meta_size) == self._meta_size:
                self._meta[piece] = data        # only pieces of the announced size: bounded memory
                self._meta_src[piece] = p.key
                self._check_metadata()
            elif t == pw.META_REJECT:
                p.meta_requested = False

    def _request_metadata(self, p: _Peer) -> None:
        if self.info is not None or not self._meta_size or p.meta_requested or not p.ext:
            return
        if p.key in self._meta_bad or p.ext.metadata_size != self._meta_size:
            return                          # a peer that lied, or one announcing other metadata
        their = p.ext.m.get("ut_metadata")
        if not their:
            return
        if self._meta_single:
            now = time.monotonic()
            for q in self.peers.values():
                if q is not p and q.meta_requested and now - q.meta_asked_at > 15.0:
                    q.meta_requested = False      # a silent source does not hold the others back
            if any(q.meta_requested for q in self.peers.values() if q is not p):
                return                      # one source at a time until the culprit is known
        p.meta_requested = True
        p.meta_asked_at = time.monotonic()
        for k in range(-(-self._meta_size // BLOCK)):
            if k not in self._meta:
                p.wire.extended(their, pw.meta_msg(pw.META_REQUEST, k))

    def _check_metadata(self) -> None:
        if self._meta_size is None:
            return
        n = -(-self._meta_size // BLOCK)
        if len(self._meta) < n or any(k not in self._meta for k in range(n)):
            return
        raw = b"".join(self._meta[k] for k in range(n))[:self._meta_size]
        if hashlib.sha1(raw).digest() != self.infohash and hashlib.sha256(raw).digest()[:20] != self.infohash:
            self._metadata_failed("received metadata does not match info-hash")
            return
        try:
            info = Info.parse(raw)
        except MetainfoError as e:
            self._metadata_failed(f"bad metadata: {e}")
            return
        self._set_info(info)
        for p in self.peers.values():
            pend = getattr(p, "pending_bitfield", None)
            if pend is not None:
                try:
                    self._peer_has(p, sorted(pw.bits_to_set(pend, info.num_pieces)))
                except pw.PeerError:
                    p.wire.close()           # its early bitfield does not fit the torrent: drop it
                    continue
            if getattr(p, "pending_have_all", False):
                self._peer_has(p, range(info.num_pieces))

    def _metadata_failed(self, why: str) -> None:
        """Assembled metadata failed the info-hash.  A sole contributor lied:
        it is never asked again (anacrolix drops such a peer).  Several: the
        pieces are fetched again one peer at a time, so the next failure has
        one contributor.  The size to assemble is re-chosen from the peers not
        known to lie (the liar may be the one whose size was taken)."""
        srcs = set(self._meta_src.values())
        if len(srcs) == 1:
            self._meta_bad |= srcs
        else:
            self._meta_single = True
        log.with_fields(contributors=len(srcs), liars=len(self._meta_bad)).warn("%s; retrying", why)
        self._meta.clear()
        self._meta_src.clear()
        sizes = collections.Counter(q.ext.metadata_size for q in self.peers.values()
                                    if q.ext and q.key not in self._meta_bad and "ut_metadata" in q.ext.m
                                    and q.ext.metadata_size and 0 < q.ext.metadata_size < 16 * 1024 * 1024)
        self._meta_size = sizes.most_common(1)[0][0] if sizes else None
        for q in self.peers.values():
            q.meta_requested = False
            self._request_metadata(q)
