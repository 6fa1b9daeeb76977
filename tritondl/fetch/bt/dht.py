"""Mainline DHT (BEP 5) with IPv6 (BEP 32) — KRPC over UDP.

What anacrolix's default client runs for the reference
(``internal/downloader/torrent/torrent.go:40-48`` ``NewDefaultClientConfig``
→ a DHT server on IPv4 and IPv6), and what makes a bare ``magnet:?xt=``
resolve on the real internet:

* **routing table** — 160 distance buckets of ``K = 8`` nodes each (bucket
  ``b`` holds ids whose XOR distance to ours has bit length ``b + 1``) with
  a replacement cache.  A full bucket never drops a node on hearsay: a node
  that failed twice is *bad* and is replaced at once; otherwise the
  least-recently-seen *questionable* node (silent for ``stale_after``,
  15 min) is pinged, and only if it fails to answer twice is it evicted in
  favour of the newest replacement — BEP 5 "ping before evict".  Buckets idle
  for ``refresh_after`` are refreshed with a lookup of a random id in range;
* **iterative lookup** — ``α = 3`` queries in flight toward the target,
  keeping a shortlist ordered by XOR distance; it ends when the ``2K``
  closest nodes that have not failed have all answered (convergence), not
  after a fixed number of rounds; the K closest of them are the result.  Timeouts mark the node failed in the
  table.  Each lookup's query/response/timeout counts land in
  :attr:`DHTNode.last_lookup`;
* **server side** — answers ``ping``/``find_node``/``get_peers``/
  ``announce_peer``; tokens are an HMAC-like hash of the querier's IP under a
  secret rotated every ``token_rotate`` (5 min) — the current and previous
  secrets are accepted, as BEP 5 recommends; announced peers expire after
  30 min;
* **BEP 32** — one socket and one routing table per address family;
  ``nodes6`` (38-byte entries) and 18-byte IPv6 ``values``; the ``want``
  argument (``n4``/``n6``) selects which node lists a reply carries;
  lookups run per family and ``get_peers`` merges them;
* **announce** — after a ``get_peers`` lookup, ``announce_peer`` goes to the
  ``K`` closest nodes (per family) that returned a token.
"""

from __future__ import annotations

import asyncio
import collections
import hashlib
import ipaddress
import os
import random
import socket
import struct
import time
from dataclasses import dataclass, field
from typing import Iterable

from ...utils.log import log
from . import bencode

K = 8
LOOKUP_MAX_VALUES_PER_REPLY = 500    # BEP 5 replies fit a datagram: ~250 compact IPv4 peers at 1500 B
LOOKUP_MAX_PEERS = 5000              # peers one get_peers lookup collects (the torrent keeps 500)
ALPHA = 3
ID_BITS = 160


def xor_distance(a: bytes, b: bytes) -> int:
    return int.from_bytes(a, "big") ^ int.from_bytes(b, "big")


def _is_v6(host: str) -> bool:
    return ":" in host


def compact_addr(addr: tuple[str, int]) -> bytes:
    if _is_v6(addr[0]):
        return socket.inet_pton(socket.AF_INET6, addr[0]) + struct.pack(">H", addr[1])
    return socket.inet_aton(addr[0]) + struct.pack(">H", addr[1])


def compact_node(nid: bytes, addr: tuple[str, int]) -> bytes:
    return nid + compact_addr(addr)


def parse_nodes(b: bytes) -> list[tuple[bytes, tuple[str, int]]]:
    """BEP 5 ``nodes``: 26-byte entries (id, IPv4, port)."""
    out = []
    for i in range(0, len(b) - 25, 26):
        nid = b[i:i + 20]
        ip = socket.inet_ntoa(b[i + 20:i + 24])
        (port,) = struct.unpack(">H", b[i + 24:i + 26])
        if port:
            out.append((nid, (ip, port)))
    return out


def parse_nodes6(b: bytes) -> list[tuple[bytes, tuple[str, int]]]:
    """BEP 32 ``nodes6``: 38-byte entries (id, IPv6, port)."""
    out = []
    for i in range(0, len(b) - 37, 38):
        nid = b[i:i + 20]
        ip = socket.inet_ntop(socket.AF_INET6, b[i + 20:i + 36])
        (port,) = struct.unpack(">H", b[i + 36:i + 38])
        if port:
            out.append((nid, (ip, port)))
    return out


def parse_values(vals: Iterable) -> list[tuple[str, int]]:
    """Compact peers: 6-byte IPv4 and (BEP 32) 18-byte IPv6 entries."""
    out = []
    for v in vals:
        if not isinstance(v, bytes):
            continue
        if len(v) == 6:
            out.append((socket.inet_ntoa(v[:4]), struct.unpack(">H", v[4:])[0]))
        elif len(v) == 18:
            out.append((socket.inet_ntop(socket.AF_INET6, v[:16]), struct.unpack(">H", v[16:])[0]))
    return out


def bucket_index(own: bytes, nid: bytes) -> int:
    """Distance bucket: bit length of XOR distance minus one (0..159)."""
    return max(0, xor_distance(own, nid).bit_length() - 1)


def random_id_in_bucket(own: bytes, b: int) -> bytes:
    """A random id whose distance to ``own`` has bit length ``b + 1``."""
    d = (1 << b) | random.getrandbits(b) if b else 1
    return (int.from_bytes(own, "big") ^ d).to_bytes(20, "big")


class KRPCError(Exception):
    pass


@dataclass
class Node:
    id: bytes
    addr: tuple[str, int]
    last_seen: float = field(default_factory=time.monotonic)
    fails: int = 0
    responded: bool = False

    @property
    def bad(self) -> bool:
        return self.fails >= 2


class RoutingTable:
    """160 distance buckets of ``k`` nodes (most recently seen last) plus a
    per-bucket replacement cache; see the module docstring for the policy."""

    def __init__(self, own_id: bytes, k: int = K, stale_after: float = 900.0) -> None:
        self.own = own_id
        self.k = k
        self.stale_after = stale_after
        self.buckets: list[list[Node]] = [[] for _ in range(ID_BITS)]
        self.replacements: list[list[Node]] = [[] for _ in range(ID_BITS)]
        self.changed = [time.monotonic()] * ID_BITS
        self._index: dict[bytes, Node] = {}

    def __len__(self) -> int:
        return len(self._index)

    def __contains__(self, nid: bytes) -> bool:
        return nid in self._index

    def get(self, nid: bytes) -> Node | None:
        return self._index.get(nid)

    def nodes(self) -> list[Node]:
        return list(self._index.values())

    def observe(self, nid: bytes, addr: tuple[str, int], responded: bool) -> Node | None:
        """Record contact with a node.  Returns a questionable node the caller
        should ping (the bucket is full of not-yet-bad nodes), else None."""
        if nid == self.own or len(nid) != 20:
            return None
        now = time.monotonic()
        n = self._index.get(nid)
        b = bucket_index(self.own, nid)
        bucket = self.buckets[b]
        if n is not None:
            n.addr, n.last_seen = addr, now
            if responded:
                n.fails, n.responded = 0, True
            bucket.remove(n)
            bucket.append(n)
            self.changed[b] = now
            return None
        node = Node(nid, addr, now, 0, responded)
        if len(bucket) < self.k:
            bucket.append(node)
            self._index[nid] = node
            self.changed[b] = now
            return None
        for i, old in enumerate(bucket):
            if old.bad:                          # a bad node is replaced outright
                del bucket[i]
                del self._index[old.id]
                bucket.append(node)
                self._index[nid] = node
                self.changed[b] = now
                return None
        repl = self.replacements[b]
        repl[:] = [r for r in repl if r.id != nid][-(self.k - 1):] + [node]
        stale = [o for o in bucket if now - o.last_seen >= self.stale_after]
        return min(stale, key=lambda o: o.last_seen) if stale else None

    def failed(self, nid: bytes) -> None:
        """A query to nid timed out.  A bad node with a replacement waiting is
        swapped out right away."""
        n = self._index.get(nid)
        if n is None:
            return
        n.fails += 1
        if n.bad:
            b = bucket_index(self.own, nid)
            if self.replacements[b]:
                self.evict(nid)

    def evict(self, nid: bytes) -> None:
        n = self._index.pop(nid, None)
        if n is None:
            return
        b = bucket_index(self.own, nid)
        self.buckets[b].remove(n)
        repl = self.replacements[b]
        while repl and len(self.buckets[b]) < self.k:
            r = repl.pop()                       # newest candidate first
            if r.id not in self._index and r.id != self.own:
                self.buckets[b].append(r)
                self._index[r.id] = r
        self.changed[b] = time.monotonic()

    def closest(self, target: bytes, n: int = K) -> list[Node]:
        cand = [x for x in self._index.values() if not x.bad]
        cand.sort(key=lambda x: xor_distance(x.id, target))
        return cand[:n]

    def stale_buckets(self, refresh_after: float) -> list[int]:
        now = time.monotonic()
        return [b for b in range(ID_BITS) if self.buckets[b] and now - self.changed[b] >= refresh_after]


class _Proto(asyncio.DatagramProtocol):
    def __init__(self, node: "DHTNode", fam: int) -> None:
        self.node = node
        self.fam = fam

    def datagram_received(self, data: bytes, addr) -> None:
        self.node._on_datagram(data, (addr[0], addr[1]), self.fam)

    def error_received(self, exc) -> None:  # ICMP unreachable etc.: the query times out
        pass


def _norm_host(h: str) -> str:
    try:
        return str(ipaddress.ip_address(h.split("%")[0]))
    except ValueError:
        return h


class DHTNode:
    """One DHT participant (client + server), dual-stack when ``host6`` is set.

    ``host``/``port``: IPv4 socket (``host=None`` disables IPv4);
    ``host6``: IPv6 bind address (e.g. ``"::"``) or None; both families
    share the node id.  ``bootstrap``: (host, port) routers of either family."""

    def __init__(self, node_id: bytes | None = None, host: str | None = "0.0.0.0", port: int = 0,
                 bootstrap: list[tuple[str, int]] | None = None, timeout: float = 2.0, *,
                 host6: str | None = None, port6: int = 0, k: int = K, alpha: int = ALPHA,
                 stale_after: float = 900.0, refresh_after: float = 900.0, token_rotate: float = 300.0,
                 peer_ttl: float = 1800.0, max_lookup_queries: int = 400, lookup_width: int = 0,
                 max_torrents: int = 2000, max_peers_per_torrent: int = 2000) -> None:
        self.id = node_id or hashlib.sha1(os.urandom(20)).digest()
        # announce_peer store bounds (libtorrent dht_max_torrents / dht_max_peers): the
        # least recently announced info-hash is evicted first, and expired peers and
        # empty info-hashes are purged by the maintenance loop, so a long-running
        # worker's DHT memory stays bounded whatever announces it receives
        self.max_torrents = max_torrents
        self.max_peers_per_torrent = max_peers_per_torrent
        self.host, self.port = host, port
        self.host6, self.port6 = host6, port6
        self.bootstrap_nodes = list(bootstrap or [])
        self.timeout = timeout
        self.k, self.alpha = k, alpha
        self.refresh_after = refresh_after
        self.token_rotate = token_rotate
        self.peer_ttl = peer_ttl
        self.max_lookup_queries = max_lookup_queries
        # a lookup has converged when the `lookup_width` closest live nodes have all
        # answered (default 2K): exploring wider than the K it reports/announces to
        # keeps a lookup from settling on a local minimum of incomplete routing
        # tables, so announcer and searcher reliably meet on the same K nodes
        self.lookup_width = lookup_width or 2 * k
        self.tables = {socket.AF_INET: RoutingTable(self.id, k, stale_after),
                       socket.AF_INET6: RoutingTable(self.id, k, stale_after)}
        self.peers: dict[bytes, dict[tuple[str, int], float]] = {}
        self._pending: dict[bytes, tuple[tuple[str, int], asyncio.Future]] = {}
        self._tid = random.getrandbits(16)
        self._secret = os.urandom(16)
        self._old_secret = self._secret
        self._secret_t = time.monotonic()
        self._transports: dict[int, asyncio.DatagramTransport] = {}
        self._pinging: set[bytes] = set()
        self._tasks: set[asyncio.Task] = set()
        self.last_lookup: dict = {}
        self.lookups: collections.deque = collections.deque(maxlen=64)     # recent lookup stats
        self.last_closest: list[tuple[bytes, tuple[str, int]]] = []
        self.stats = {"queries_sent": 0, "responses": 0, "timeouts": 0, "queries_served": 0, "evicted": 0}

    # ------------------------------------------------------------ lifecycle
    async def start(self, maintain: bool = False) -> "DHTNode":
        loop = asyncio.get_running_loop()
        if self.host is not None:
            tr, _ = await loop.create_datagram_endpoint(lambda: _Proto(self, socket.AF_INET),
                                                        local_addr=(self.host, self.port), family=socket.AF_INET)
            self._transports[socket.AF_INET] = tr
            self.port = tr.get_extra_info("sockname")[1]
        if self.host6 is not None:
            try:
                tr6, _ = await loop.create_datagram_endpoint(lambda: _Proto(self, socket.AF_INET6),
                                                             local_addr=(self.host6, self.port6),
                                                             family=socket.AF_INET6)
                self._transports[socket.AF_INET6] = tr6
                self.port6 = tr6.get_extra_info("sockname")[1]
            except OSError as e:
                log.with_field("error", str(e)).warn("dht: IPv6 socket unavailable; IPv4 only")
        if maintain:
            self._spawn(self._maintain())
        return self

    def stop(self) -> None:
        for tr in self._transports.values():
            tr.close()
        self._transports.clear()
        for _addr, f in self._pending.values():
            if not f.done():
                f.cancel()
        self._pending.clear()
        for t in list(self._tasks):
            t.cancel()

    def _spawn(self, coro) -> asyncio.Task:
        t = asyncio.ensure_future(coro)
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)
        return t

    @property
    def addr(self) -> tuple[str, int]:
        return ("127.0.0.1" if self.host in ("0.0.0.0", "", None) else self.host, self.port)

    @property
    def addr6(self) -> tuple[str, int] | None:
        if socket.AF_INET6 not in self._transports:
            return None
        return ("::1" if self.host6 in ("::", "") else self.host6, self.port6)

    @property
    def families(self) -> list[int]:
        return list(self._transports)

    @property
    def table(self) -> RoutingTable:
        """The IPv4 routing table (BEP 5)."""
        return self.tables[socket.AF_INET]

    @property
    def table6(self) -> RoutingTable:
        return self.tables[socket.AF_INET6]

    # ------------------------------------------------------------ table
    def add_node(self, nid: bytes, addr: tuple[str, int], responded: bool = False) -> None:
        fam = socket.AF_INET6 if _is_v6(addr[0]) else socket.AF_INET
        q = self.tables[fam].observe(nid, addr, responded)
        if q is not None and q.id not in self._pinging and fam in self._transports:
            self._pinging.add(q.id)
            self._spawn(self._ping_or_evict(fam, q))

    async def _ping_or_evict(self, fam: int, n: Node) -> None:
        """BEP 5: a full bucket pings its least-recently-seen questionable
        node (twice) before evicting it for the newest replacement."""
        try:
            for _ in range(2):
                try:
                    await self.query(n.addr, "ping", {}, nid=n.id)
                    return                                   # alive: keep it, drop the candidate
                except (KRPCError, asyncio.TimeoutError, OSError):
                    continue
            self.tables[fam].evict(n.id)
            self.stats["evicted"] += 1
        finally:
            self._pinging.discard(n.id)

    def closest(self, target: bytes, n: int = K, fam: int = socket.AF_INET) -> list[tuple[bytes, tuple[str, int]]]:
        return [(x.id, x.addr) for x in self.tables[fam].closest(target, n)]

    def _token(self, ip: str, secret: bytes | None = None) -> bytes:
        now = time.monotonic()
        if now - self._secret_t >= self.token_rotate:
            self._old_secret, self._secret, self._secret_t = self._secret, os.urandom(16), now
        return hashlib.sha1((secret or self._secret) + _norm_host(ip).encode()).digest()[:8]

    def rotate_secret(self) -> None:
        self._old_secret, self._secret, self._secret_t = self._secret, os.urandom(16), time.monotonic()

    # ------------------------------------------------------------ wire
    def _send(self, msg: dict, addr: tuple[str, int]) -> None:
        fam = socket.AF_INET6 if _is_v6(addr[0]) else socket.AF_INET
        tr = self._transports.get(fam)
        if tr is not None:
            tr.sendto(bencode.encode(msg), addr)

    def _on_datagram(self, data: bytes, addr: tuple[str, int], fam: int) -> None:
        try:
            msg = bencode.decode(data)
        except bencode.BencodeError:
            return
        if not isinstance(msg, dict):
            return
        y = msg.get(b"y")
        t = msg.get(b"t", b"")
        if not isinstance(t, bytes):
            return                                           # transaction ids are strings (BEP 5)
        if y == b"q":
            self._on_query(msg, t, addr, fam)
        elif y in (b"r", b"e"):
            ent = self._pending.get(t)
            if ent is None:
                return
            want_addr, f = ent
            if (_norm_host(want_addr[0]), want_addr[1]) != (_norm_host(addr[0]), addr[1]):
                return                                       # not who we asked: ignore (anti-spoof)
            self._pending.pop(t, None)
            if f.done():
                return
            if y == b"r":
                r = msg.get(b"r")
                if not isinstance(r, dict):
                    f.set_exception(KRPCError("malformed response"))
                    return
                nid = r.get(b"id")
                if isinstance(nid, bytes) and len(nid) == 20:
                    self.add_node(nid, addr, responded=True)
                f.set_result(r)
            else:
                f.set_exception(KRPCError(repr(msg.get(b"e"))))

    def _nodes_for(self, target: bytes, want: set, fam: int) -> dict:
        out: dict = {}
        if b"n4" in want or (not want and fam == socket.AF_INET):
            out[b"nodes"] = b"".join(compact_node(n.id, n.addr) for n in self.tables[socket.AF_INET].closest(target))
        if b"n6" in want or (not want and fam == socket.AF_INET6):
            out[b"nodes6"] = b"".join(compact_node(n.id, n.addr)
                                      for n in self.tables[socket.AF_INET6].closest(target))
        return out

    def _on_query(self, msg: dict, t: bytes, addr: tuple[str, int], fam: int) -> None:
        q = msg.get(b"q")
        a = msg.get(b"a")
        if not isinstance(a, dict):
            self._send({b"t": t, b"y": b"e", b"e": [203, b"missing arguments"]}, addr)
            return
        self.stats["queries_served"] += 1
        nid = a.get(b"id")
        if isinstance(nid, bytes) and len(nid) == 20:
            self.add_node(nid, addr)
        w = a.get(b"want")
        want = {x for x in w if isinstance(x, bytes)} if isinstance(w, list) else set()
        r: dict = {b"id": self.id}
        if q == b"ping":
            pass
        elif q == b"find_node":
            target = a.get(b"target", b"")
            if not isinstance(target, bytes) or len(target) != 20:
                self._send({b"t": t, b"y": b"e", b"e": [203, b"bad target"]}, addr)
                return
            r.update(self._nodes_for(target, want, fam))
        elif q == b"get_peers":
            ih = a.get(b"info_hash", b"")
            if not isinstance(ih, bytes) or len(ih) != 20:
                self._send({b"t": t, b"y": b"e", b"e": [203, b"bad info_hash"]}, addr)
                return
            r[b"token"] = self._token(addr[0])
            peers = self._live_peers(ih)
            fam_peers = [p for p in peers if _is_v6(p[0]) == (fam == socket.AF_INET6)]
            if fam_peers:
                random.shuffle(fam_peers)
                r[b"values"] = [compact_addr(p) for p in fam_peers[:50]]
            r.update(self._nodes_for(ih, want, fam))
        elif q == b"announce_peer":
            ih = a.get(b"info_hash", b"")
            tok = a.get(b"token", b"")
            if not isinstance(ih, bytes) or len(ih) != 20 or \
                    tok not in (self._token(addr[0]), self._token(addr[0], self._old_secret)):
                self._send({b"t": t, b"y": b"e", b"e": [203, b"bad token"]}, addr)
                return
            port = addr[1] if a.get(b"implied_port") else a.get(b"port", 0)
            if not isinstance(port, int) or not 0 < port < 65536:
                self._send({b"t": t, b"y": b"e", b"e": [203, b"bad port"]}, addr)
                return
            self._store_peer(ih, (_norm_host(addr[0]), int(port)))
        else:
            self._send({b"t": t, b"y": b"e", b"e": [204, b"method unknown"]}, addr)
            return
        self._send({b"t": t, b"y": b"r", b"r": r}, addr)

    def _store_peer(self, ih: bytes, peer: tuple[str, int]) -> None:
        """Record an announce.  ``self.peers`` is kept in announce order (an
        info-hash moves to the end on every announce), so the first key is the
        least recently announced one — evicted when the store is full."""
        store = self.peers.pop(ih, None)
        if store is None:
            store = {}
            while len(self.peers) >= self.max_torrents:
                del self.peers[next(iter(self.peers))]
        self.peers[ih] = store
        store.pop(peer, None)
        store[peer] = time.monotonic()          # dict order == announce order
        while len(store) > self.max_peers_per_torrent:
            del store[next(iter(store))]

    def purge_peers(self) -> int:
        """Drop expired announces and info-hashes left with none; returns how
        many info-hashes were removed."""
        cutoff = time.monotonic() - self.peer_ttl
        gone = 0
        for ih in list(self.peers):
            store = self.peers[ih]
            while store:
                first = next(iter(store))
                if store[first] >= cutoff:
                    break                       # announce order: the rest are newer
                del store[first]
            if not store:
                del self.peers[ih]
                gone += 1
        return gone

    def _live_peers(self, ih: bytes) -> list[tuple[str, int]]:
        store = self.peers.get(ih)
        if not store:
            return []
        cutoff = time.monotonic() - self.peer_ttl
        for p in [p for p, ts in store.items() if ts < cutoff]:
            del store[p]
        return list(store)

    async def query(self, addr: tuple[str, int], q: str, args: dict, nid: bytes | None = None,
                    want: list[bytes] | None = None) -> dict:
        self._tid = (self._tid + 1) & 0xFFFF
        t = struct.pack(">H", self._tid)
        fut = asyncio.get_running_loop().create_future()
        self._pending[t] = (addr, fut)
        a = {b"id": self.id, **args}
        if want:
            a[b"want"] = want
        self.stats["queries_sent"] += 1
        self._send({b"t": t, b"y": b"q", b"q": q.encode(), b"a": a}, addr)
        try:
            r = await asyncio.wait_for(fut, self.timeout)
            self.stats["responses"] += 1
            return r
        except asyncio.TimeoutError:
            self.stats["timeouts"] += 1
            if nid is not None:
                self.tables[socket.AF_INET6 if _is_v6(addr[0]) else socket.AF_INET].failed(nid)
            raise
        finally:
            if self._pending.get(t, (None, None))[1] is fut:
                del self._pending[t]

    # ------------------------------------------------------------ client ops
    def _fam_of(self, addr: tuple[str, int]) -> int:
        return socket.AF_INET6 if _is_v6(addr[0]) else socket.AF_INET

    async def _routers(self, fam: int) -> list[tuple[str, int]]:
        """Bootstrap routers of this family; host names (``router.bittorrent.com``)
        resolve to every address of the family (replies are matched by address)."""
        loop = asyncio.get_running_loop()
        out: list[tuple[str, int]] = []
        for host, port in self.bootstrap_nodes:
            try:
                ipaddress.ip_address(host.split("%")[0])
                if self._fam_of((host, port)) == fam:
                    out.append((host, port))
                continue
            except ValueError:
                pass
            try:
                infos = await loop.getaddrinfo(host, port, family=fam, type=socket.SOCK_DGRAM)
            except (OSError, UnicodeError):
                continue
            for _f, _t, _p, _c, sa in infos:
                if (sa[0], sa[1]) not in out:
                    out.append((sa[0], sa[1]))
        return out

    async def _ask_routers(self, target: bytes, fam: int) -> None:
        """Query the bootstrap routers of this family (ids unknown) to seed the table."""
        routers = await self._routers(fam)

        async def one(addr):
            try:
                r = await self.query(addr, "find_node", {b"target": target})
            except (KRPCError, asyncio.TimeoutError, OSError) as e:
                log.with_fields(node=f"{addr[0]}:{addr[1]}", error=str(e)).debug("dht bootstrap node failed")
                return
            for nid, a in self._parse_reply_nodes(r, fam):
                self.add_node(nid, a)
        await asyncio.gather(*(one(a) for a in routers))

    def _parse_reply_nodes(self, r: dict, fam: int) -> list[tuple[bytes, tuple[str, int]]]:
        if fam == socket.AF_INET6:
            v = r.get(b"nodes6", b"")
            return parse_nodes6(v) if isinstance(v, bytes) else []
        v = r.get(b"nodes", b"")
        return parse_nodes(v) if isinstance(v, bytes) else []

    async def bootstrap(self) -> int:
        """Join: ask the routers, then look up our own id (fills the buckets
        near us, and tells those nodes about us)."""
        for fam in self.families:
            await self._ask_routers(self.id, fam)
            if len(self.tables[fam]):
                await self._lookup(self.id, "find_node", fam)
        return sum(len(self.tables[f]) for f in self.families)

    async def refresh(self) -> int:
        """Look up a random id in every bucket idle for ``refresh_after``."""
        n = 0
        for fam in self.families:
            for b in self.tables[fam].stale_buckets(self.refresh_after):
                await self._lookup(random_id_in_bucket(self.id, b), "find_node", fam)
                n += 1
        return n

    async def _maintain(self) -> None:
        period = max(1.0, min(60.0, self.refresh_after / 4))
        while True:
            await asyncio.sleep(period)
            self.purge_peers()
            try:
                await self.refresh()
            except Exception as e:  # noqa: BLE001 - maintenance must not die
                log.with_field("error", str(e)).debug("dht refresh failed")

    async def find_node(self, target: bytes, fam: int = socket.AF_INET) -> list[tuple[bytes, tuple[str, int]]]:
        """The K closest live nodes to ``target`` (iterative, to convergence)."""
        await self._lookup(target, "find_node", fam)
        return list(self.last_closest)

    async def get_peers(self, infohash: bytes, max_rounds: int | None = None) -> list[tuple[str, int]]:
        """Peers for ``infohash`` from every family's lookup (``max_rounds``
        is accepted for compatibility; lookups end on convergence)."""
        res = await asyncio.gather(*(self._lookup(infohash, "get_peers", f) for f in self.families))
        found: list[tuple[str, int]] = []
        for peers, _tok in res:
            for p in peers:
                if p not in found:
                    found.append(p)
        return found

    async def announce_peer(self, infohash: bytes, port: int) -> int:
        """Announce to the K closest token-granting nodes of each family."""
        ok = 0
        for fam in self.families:
            _found, tokens = await self._lookup(infohash, "get_peers", fam)
            best = sorted(tokens.items(), key=lambda kv: xor_distance(kv[0], infohash))[:self.k]

            async def one(nid, addr, tok):
                try:
                    await self.query(addr, "announce_peer", {b"info_hash": infohash, b"port": port, b"token": tok,
                                                             b"implied_port": 0}, nid=nid)
                    return 1
                except (KRPCError, asyncio.TimeoutError, OSError):
                    return 0
            ok += sum(await asyncio.gather(*(one(nid, a, tok) for nid, (a, tok) in best)))
        return ok

    async def _lookup(self, target: bytes, method: str, fam: int = socket.AF_INET):
        """Iterative lookup until the K closest live nodes have all answered.
        Returns (peers, {node id: (addr, token)})."""
        table = self.tables[fam]
        arg = {b"info_hash": target} if method == "get_peers" else {b"target": target}
        want = [b"n6"] if fam == socket.AF_INET6 else [b"n4"]
        if not len(table):
            await self._ask_routers(target, fam)
        known: dict[bytes, tuple[str, int]] = {n.id: n.addr for n in table.closest(target, 2 * self.lookup_width)}
        state: dict[bytes, str] = {nid: "new" for nid in known}       # new | wait | ok | dead
        found: list[tuple[str, int]] = []
        seen: set[tuple[str, int]] = set()
        tokens: dict[bytes, tuple[tuple[str, int], bytes]] = {}
        inflight: dict[asyncio.Task, bytes] = {}
        st = {"queries": 0, "responses": 0, "timeouts": 0}

        def order() -> list[bytes]:
            return sorted((nid for nid, s in state.items() if s != "dead"),
                          key=lambda nid: xor_distance(nid, target))

        try:
            while True:
                top = order()[:self.lookup_width]
                if all(state[nid] == "ok" for nid in top) and not any(state[n] == "wait" for n in top):
                    break                                                   # converged
                for nid in top:
                    if len(inflight) >= self.alpha or st["queries"] >= self.max_lookup_queries:
                        break
                    if state[nid] == "new":
                        state[nid] = "wait"
                        st["queries"] += 1
                        t = asyncio.ensure_future(self.query(known[nid], method, arg, nid=nid, want=want))
                        inflight[t] = nid
                if not inflight:
                    break                                    # query budget spent, or nothing left to ask
                done, _ = await asyncio.wait(inflight, return_when=asyncio.FIRST_COMPLETED)
                for t in done:
                    nid = inflight.pop(t)
                    exc = t.exception()
                    if exc is not None:
                        state[nid] = "dead"
                        st["timeouts"] += isinstance(exc, asyncio.TimeoutError)
                        continue
                    r = t.result()
                    st["responses"] += 1
                    rid = r.get(b"id")
                    if isinstance(rid, bytes) and rid != nid:
                        state[nid] = "dead"                  # answered with another identity
                        continue
                    state[nid] = "ok"
                    tok = r.get(b"token")
                    if isinstance(tok, bytes):
                        tokens[nid] = (known[nid], tok)
                    vals = r.get(b"values")
                    if isinstance(vals, list):
                        # a datagram can carry thousands of values or nodes: take what an
                        # honest node sends (values up to the lookup's cap, K nodes)
                        for p in parse_values(vals[:LOOKUP_MAX_VALUES_PER_REPLY]):
                            if p not in seen and len(found) < LOOKUP_MAX_PEERS:
                                seen.add(p)
                                found.append(p)
                    for cid, ca in self._parse_reply_nodes(r, fam)[:2 * K]:
                        if cid == self.id or cid in state:
                            continue
                        known[cid] = ca
                        state[cid] = "new"
        finally:
            for t in inflight:
                t.cancel()
        top = order()[:self.lookup_width]
        st.update(target=target.hex(), method=method, family="ipv6" if fam == socket.AF_INET6 else "ipv4",
                  peers=len(found), converged=all(state[n] == "ok" for n in top))
        self.last_lookup = st
        self.lookups.append(st)
        self.last_closest = [(nid, known[nid]) for nid in top if state[nid] == "ok"][:self.k]
        log.with_fields(**{k: v for k, v in st.items() if k != "target"}).debug("dht lookup done")
        return found, tokens
