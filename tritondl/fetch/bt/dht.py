"""Mainline DHT (BEP 5) — KRPC over UDP.

Client side: iterative ``get_peers`` lookup (α = 3 parallel queries toward
the info-hash by XOR distance) and ``announce_peer``.  Server side: answers
``ping`` / ``find_node`` / ``get_peers`` / ``announce_peer`` so that a set of
nodes forms a working DHT (used by the test swarm; anacrolix runs a full DHT
server by default, which is what makes bare ``magnet:?xt=`` links work).
"""

from __future__ import annotations

import asyncio
import hashlib
import os
import socket
import struct
import time
from typing import Iterable

from ...utils.log import log
from . import bencode

K = 8


def xor_distance(a: bytes, b: bytes) -> int:
    return int.from_bytes(a, "big") ^ int.from_bytes(b, "big")


def compact_node(nid: bytes, addr: tuple[str, int]) -> bytes:
    return nid + socket.inet_aton(addr[0]) + struct.pack(">H", addr[1])


def parse_nodes(b: bytes) -> list[tuple[bytes, tuple[str, int]]]:
    out = []
    for i in range(0, len(b) - 25, 26):
        nid = b[i:i + 20]
        ip = socket.inet_ntoa(b[i + 20:i + 24])
        (port,) = struct.unpack(">H", b[i + 24:i + 26])
        if port:
            out.append((nid, (ip, port)))
    return out


def parse_values(vals: Iterable) -> list[tuple[str, int]]:
    out = []
    for v in vals:
        if isinstance(v, bytes) and len(v) == 6:
            out.append((socket.inet_ntoa(v[:4]), struct.unpack(">H", v[4:])[0]))
    return out


class KRPCError(Exception):
    pass


class _Proto(asyncio.DatagramProtocol):
    def __init__(self, node: "DHTNode") -> None:
        self.node = node

    def datagram_received(self, data: bytes, addr) -> None:
        self.node._on_datagram(data, addr)


class DHTNode:
    def __init__(self, node_id: bytes | None = None, host: str = "0.0.0.0", port: int = 0,
                 bootstrap: list[tuple[str, int]] | None = None, timeout: float = 2.0) -> None:
        self.id = node_id or hashlib.sha1(os.urandom(20)).digest()
        self.host, self.port = host, port
        self.bootstrap_nodes = bootstrap or []
        self.timeout = timeout
        self.table: dict[bytes, tuple[tuple[str, int], float]] = {}
        self.peers: dict[bytes, dict[tuple[str, int], float]] = {}
        self._pending: dict[bytes, asyncio.Future] = {}
        self._tid = 0
        self._secret = os.urandom(16)
        self._old_secret = self._secret
        self.transport: asyncio.DatagramTransport | None = None
        self.max_table = 8 * 160

    # ------------------------------------------------------------ lifecycle
    async def start(self) -> "DHTNode":
        loop = asyncio.get_running_loop()
        self.transport, _ = await loop.create_datagram_endpoint(lambda: _Proto(self),
                                                                local_addr=(self.host, self.port))
        self.port = self.transport.get_extra_info("sockname")[1]
        return self

    def stop(self) -> None:
        if self.transport is not None:
            self.transport.close()
            self.transport = None
        for f in self._pending.values():
            if not f.done():
                f.cancel()
        self._pending.clear()

    @property
    def addr(self) -> tuple[str, int]:
        return ("127.0.0.1" if self.host in ("0.0.0.0", "") else self.host, self.port)

    # ------------------------------------------------------------ table
    def add_node(self, nid: bytes, addr: tuple[str, int]) -> None:
        if nid == self.id or len(nid) != 20:
            return
        self.table[nid] = (addr, time.monotonic())
        if len(self.table) > self.max_table:
            oldest = min(self.table, key=lambda k: self.table[k][1])
            self.table.pop(oldest, None)

    def closest(self, target: bytes, n: int = K) -> list[tuple[bytes, tuple[str, int]]]:
        return [(nid, a) for nid, (a, _t) in sorted(self.table.items(),
                                                     key=lambda kv: xor_distance(kv[0], target))[:n]]

    def _token(self, ip: str, secret: bytes | None = None) -> bytes:
        return hashlib.sha1((secret or self._secret) + ip.encode()).digest()[:8]

    # ------------------------------------------------------------ wire
    def _send(self, msg: dict, addr: tuple[str, int]) -> None:
        if self.transport is not None:
            self.transport.sendto(bencode.encode(msg), addr)

    def _on_datagram(self, data: bytes, addr: tuple[str, int]) -> None:
        try:
            msg = bencode.decode(data)
        except bencode.BencodeError:
            return
        if not isinstance(msg, dict):
            return
        y = msg.get(b"y")
        t = msg.get(b"t", b"")
        if y == b"q":
            self._on_query(msg, t, addr)
        elif y in (b"r", b"e"):
            f = self._pending.pop(t, None)
            if f is not None and not f.done():
                if y == b"r":
                    r = msg.get(b"r") or {}
                    nid = r.get(b"id")
                    if isinstance(nid, bytes):
                        self.add_node(nid, addr)
                    f.set_result(r)
                else:
                    f.set_exception(KRPCError(repr(msg.get(b"e"))))

    def _on_query(self, msg: dict, t: bytes, addr: tuple[str, int]) -> None:
        q = msg.get(b"q")
        a = msg.get(b"a") or {}
        nid = a.get(b"id")
        if isinstance(nid, bytes):
            self.add_node(nid, addr)
        r: dict = {b"id": self.id}
        if q == b"ping":
            pass
        elif q == b"find_node":
            target = a.get(b"target", b"")
            r[b"nodes"] = b"".join(compact_node(n, ad) for n, ad in self.closest(target))
        elif q == b"get_peers":
            ih = a.get(b"info_hash", b"")
            r[b"token"] = self._token(addr[0])
            peers = self.peers.get(ih)
            if peers:
                r[b"values"] = [socket.inet_aton(h) + struct.pack(">H", p) for (h, p) in list(peers)[:50]]
            r[b"nodes"] = b"".join(compact_node(n, ad) for n, ad in self.closest(ih))
        elif q == b"announce_peer":
            ih = a.get(b"info_hash", b"")
            tok = a.get(b"token", b"")
            if tok not in (self._token(addr[0]), self._token(addr[0], self._old_secret)):
                self._send({b"t": t, b"y": b"e", b"e": [203, b"bad token"]}, addr)
                return
            port = addr[1] if a.get(b"implied_port") else a.get(b"port", 0)
            self.peers.setdefault(ih, {})[(addr[0], int(port))] = time.monotonic()
        else:
            self._send({b"t": t, b"y": b"e", b"e": [204, b"method unknown"]}, addr)
            return
        self._send({b"t": t, b"y": b"r", b"r": r}, addr)

    async def query(self, addr: tuple[str, int], q: str, args: dict) -> dict:
        self._tid = (self._tid + 1) & 0xFFFF
        t = struct.pack(">H", self._tid)
        fut = asyncio.get_running_loop().create_future()
        self._pending[t] = fut
        self._send({b"t": t, b"y": b"q", b"q": q.encode(), b"a": {b"id": self.id, **args}}, addr)
        try:
            return await asyncio.wait_for(fut, self.timeout)
        finally:
            self._pending.pop(t, None)

    # ------------------------------------------------------------ client ops
    async def bootstrap(self) -> int:
        for addr in self.bootstrap_nodes:
            try:
                r = await self.query(addr, "find_node", {b"target": self.id})
                for nid, a in parse_nodes(r.get(b"nodes", b"")):
                    self.add_node(nid, a)
            except (KRPCError, asyncio.TimeoutError, OSError) as e:
                log.with_fields(node=f"{addr[0]}:{addr[1]}", error=str(e)).debug("dht bootstrap node failed")
        if self.table:
            await self._lookup(self.id, "find_node")
        return len(self.table)

    async def get_peers(self, infohash: bytes, max_rounds: int = 8) -> list[tuple[str, int]]:
        found, _tokens = await self._lookup(infohash, "get_peers", max_rounds)
        return found

    async def announce_peer(self, infohash: bytes, port: int) -> int:
        _found, tokens = await self._lookup(infohash, "get_peers")
        ok = 0
        for addr, tok in list(tokens.items())[:K]:
            try:
                await self.query(addr, "announce_peer", {b"info_hash": infohash, b"port": port, b"token": tok,
                                                         b"implied_port": 0})
                ok += 1
            except (KRPCError, asyncio.TimeoutError, OSError):
                pass
        return ok

    async def _lookup(self, target: bytes, method: str, max_rounds: int = 8):
        arg = {b"info_hash": target} if method == "get_peers" else {b"target": target}
        queried: set[tuple[str, int]] = set()
        found: list[tuple[str, int]] = []
        tokens: dict[tuple[str, int], bytes] = {}
        shortlist = self.closest(target, 3 * K) or [(b"\x00" * 20, a) for a in self.bootstrap_nodes]
        for _ in range(max_rounds):
            cand = [(n, a) for n, a in sorted(shortlist, key=lambda x: xor_distance(x[0], target))
                    if a not in queried][:3]
            if not cand:
                break
            for _n, a in cand:
                queried.add(a)
            res = await asyncio.gather(*(self.query(a, method, arg) for _n, a in cand), return_exceptions=True)
            for (_n, a), r in zip(cand, res):
                if isinstance(r, BaseException):
                    continue
                if b"token" in r:
                    tokens[a] = r[b"token"]
                for p in parse_values(r.get(b"values", [])):
                    if p not in found:
                        found.append(p)
                for nid, na in parse_nodes(r.get(b"nodes", b"")):
                    self.add_node(nid, na)
                    if all(na != x[1] for x in shortlist):
                        shortlist.append((nid, na))
        return found, tokens
