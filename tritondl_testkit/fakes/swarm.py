"""Local BitTorrent swarm for tests/benches: HTTP tracker, UDP tracker
(BEP 15), DHT nodes and seeders (our own :class:`Torrent` in seed mode) —
all on 127.0.0.1.  The reference had no swarm fixture."""

from __future__ import annotations

import asyncio
import os
import random
import struct
import time

from aiohttp import web

from tritondl.fetch.bt import bencode
from tritondl.fetch.bt.dht import DHTNode
from tritondl.fetch.bt.metainfo import Info, Magnet, Metainfo, make_info
from tritondl.fetch.bt.torrent import Torrent, TorrentConfig
from tritondl.fetch.bt.tracker import compact_peers


class HTTPTracker:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, interval: int = 5) -> None:
        self.host, self.port, self.interval = host, port, interval
        self.swarms: dict[bytes, dict[tuple[str, int], float]] = {}
        self.announces = 0
        self._runner: web.AppRunner | None = None

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}/announce"

    async def start(self) -> "HTTPTracker":
        app = web.Application()
        app.router.add_get("/announce", self._announce)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]
        return self

    async def stop(self) -> None:
        if self._runner:
            await self._runner.cleanup()

    async def _announce(self, req: web.Request) -> web.Response:
        from urllib.parse import unquote_to_bytes
        self.announces += 1
        raw = req.query_string
        q = {}
        for part in raw.split("&"):
            k, _, v = part.partition("=")
            q[k] = unquote_to_bytes(v)
        ih = q.get("info_hash", b"")
        port = int(q.get("port", b"0") or 0)
        ip = req.remote or "127.0.0.1"
        sw = self.swarms.setdefault(ih, {})
        me = (ip, port)
        if q.get("event") == b"stopped":
            sw.pop(me, None)
        elif port:
            sw[me] = time.monotonic()
        peers = [p for p in sw if p != me]
        body = bencode.encode({b"interval": self.interval, b"peers": compact_peers(peers),
                               b"complete": len(sw), b"incomplete": 0})
        return web.Response(body=body, content_type="text/plain")


class UDPTracker(asyncio.DatagramProtocol):
    def __init__(self) -> None:
        self.swarms: dict[bytes, set[tuple[str, int]]] = {}
        self.conn_ids: set[int] = set()
        self.transport: asyncio.DatagramTransport | None = None
        self.port = 0
        self.host = "127.0.0.1"

    async def start(self, host: str = "127.0.0.1", port: int = 0) -> "UDPTracker":
        loop = asyncio.get_running_loop()
        self.transport, _ = await loop.create_datagram_endpoint(lambda: self, local_addr=(host, port))
        self.port = self.transport.get_extra_info("sockname")[1]
        self.host = host
        return self

    @property
    def url(self) -> str:
        h = f"[{self.host}]" if ":" in self.host else self.host
        return f"udp://{h}:{self.port}/announce"

    def stop(self) -> None:
        if self.transport:
            self.transport.close()

    def datagram_received(self, data: bytes, addr) -> None:
        if len(data) < 16:
            return
        conn_id, action, tid = struct.unpack(">QII", data[:16])
        if action == 0 and conn_id == 0x41727101980:
            cid = random.getrandbits(63)
            self.conn_ids.add(cid)
            self.transport.sendto(struct.pack(">IIQ", 0, tid, cid), addr)  # type: ignore[union-attr]
        elif action == 1 and conn_id in self.conn_ids and len(data) >= 98:
            ih = data[16:36]
            port = struct.unpack(">H", data[96:98])[0]
            sw = self.swarms.setdefault(ih, set())
            me = (addr[0], port)
            peers = [p for p in sw if p != me]
            sw.add(me)
            v6 = ":" in addr[0]                    # BEP 15: IPv6 transport, 18-byte peers
            self.transport.sendto(struct.pack(">IIIII", 1, tid, 10, 0, len(sw)) +  # type: ignore[union-attr]
                                  compact_peers(peers, v6=v6), addr)
        else:
            self.transport.sendto(struct.pack(">II", 3, tid) + b"bad request", addr)  # type: ignore[union-attr]


class DHTNetwork:
    """``n`` in-process DHT nodes on loopback that all join through node 0
    (the one bootstrap address), like a tiny mainline DHT.  ``ipv6`` makes
    every node dual-stack (BEP 32) with node 0 reachable on ``::1`` too.
    Joins run ``join_batch`` at a time; a second pass refreshes every node's
    own neighbourhood so early joiners also learn about late ones."""

    def __init__(self, n: int = 4, *, ipv6: bool = False, timeout: float = 2.0, join_batch: int = 16) -> None:
        self.n = n
        self.ipv6 = ipv6
        self.timeout = timeout
        self.join_batch = join_batch
        self.nodes: list[DHTNode] = []

    def _node(self, boot) -> DHTNode:
        return DHTNode(host="127.0.0.1", bootstrap=boot, timeout=self.timeout,
                       host6="::1" if self.ipv6 else None)

    async def start(self) -> "DHTNetwork":
        first = await self._node(None).start()
        self.nodes = [first]
        for _ in range(self.n - 1):
            self.nodes.append(await self._node(self.bootstrap).start())
        rest = self.nodes[1:]
        for i in range(0, len(rest), self.join_batch):
            await asyncio.gather(*(nd.bootstrap() for nd in rest[i:i + self.join_batch]))
        for i in range(0, len(self.nodes), self.join_batch):
            await asyncio.gather(*(nd.bootstrap() for nd in self.nodes[i:i + self.join_batch]))
        return self

    @property
    def bootstrap(self) -> list[tuple[str, int]]:
        out = [self.nodes[0].addr]
        a6 = self.nodes[0].addr6
        if a6 is not None:
            out.append(a6)
        return out

    def kill(self, fraction: float, rng=None) -> list[DHTNode]:
        """Stop a random ``fraction`` of the nodes (never the bootstrap node):
        they vanish without a goodbye, as dead DHT peers do."""
        import random
        rng = rng or random.Random(0)
        victims = rng.sample(self.nodes[1:], int(fraction * (len(self.nodes) - 1)))
        for nd in victims:
            nd.stop()
        return victims

    def stop(self) -> None:
        for nd in self.nodes:
            nd.stop()


class _LyingInfo:
    """An Info whose raw info-dict (what BEP 9 serves and announces the size
    of) is not the one that hashes to the info-hash."""

    def __init__(self, info: Info, raw: bytes) -> None:
        self._info = info
        self.raw = raw

    def __getattr__(self, k):
        return getattr(self._info, k)


class Seeder:
    """Seed an existing file/dir: serves pieces to any peer that connects.
    ``lie_metadata``: "data" serves flipped metadata bytes of the right
    size, "size" announces and serves metadata of another size."""

    def __init__(self, info: Info, data_dir: str, *, trackers: list[str] | None = None,
                 dht_bootstrap: list[tuple[str, int]] | None = None, corrupt: bool = False,
                 encryption: str = "allow", listen_host6: str | None = None, lie_metadata: str = "") -> None:
        self.info = info
        self.data_dir = data_dir
        self.trackers = trackers or []
        self.dht_bootstrap = dht_bootstrap
        self.corrupt = corrupt
        self.encryption = encryption
        self.listen_host6 = listen_host6
        self.lie_metadata = lie_metadata
        self.torrent: Torrent | None = None
        self.dht: DHTNode | None = None

    async def start(self) -> "Seeder":
        if self.dht_bootstrap is not None:
            self.dht = await DHTNode(host="127.0.0.1", bootstrap=self.dht_bootstrap).start()
            await self.dht.bootstrap()
        cfg = TorrentConfig(listen_host="127.0.0.1", seed=True, tracker_min_interval=1.0, dht_interval=1.0,
                            verify_device="cpu", encryption=self.encryption, listen_host6=self.listen_host6,
                            native_wire=not self.corrupt)   # corrupt: served by the patched Python path
        t = Torrent(self.info.infohash, self.data_dir, cfg, info=self.info, trackers=self.trackers, dht=self.dht)
        await t.start()
        await t.download_all()
        assert t.complete.is_set(), "seeder data does not verify"
        if self.corrupt:
            def bad(p, pl):  # serve every block with its bytes flipped
                i, off, n = struct.unpack(">III", pl[:12])
                data = t.storage.read(i, off, n)
                p.wire.piece(i, off, bytes(x ^ 0xFF for x in data))
            t._on_request = bad  # type: ignore[assignment]
        if self.lie_metadata:
            raw = self.info.raw
            bad_raw = bytes(x ^ 0x5A for x in raw) if self.lie_metadata == "data" else raw + b"x" * 40000
            t.info = _LyingInfo(t.info, bad_raw)  # type: ignore[assignment]
        self.torrent = t
        return self

    @property
    def addr(self) -> tuple[str, int]:
        assert self.torrent is not None
        return ("127.0.0.1", self.torrent.port)

    async def stop(self) -> None:
        if self.torrent is not None:
            await self.torrent.close()
        if self.dht is not None:
            self.dht.stop()


def make_payload(root: str, files: dict[str, int], seed: int = 7) -> None:
    import numpy as np
    rng = np.random.default_rng(seed)
    for rel, n in files.items():
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        rng.integers(0, 256, n, dtype=np.uint8).tofile(p)


def torrent_for(path: str, piece_length: int = 256 * 1024) -> Info:
    return make_info(path, piece_length)


def magnet_for(info: Info, trackers: list[str] | None = None, peers: list[tuple[str, int]] | None = None,
               web_seeds: list[str] | None = None) -> str:
    return Magnet(info.infohash, info.name, trackers or [], peers or [], web_seeds or []).uri()


def torrent_file_bytes(info: Info, trackers: list[str] | None = None, url_list: list[str] | None = None) -> bytes:
    return Metainfo(info, [[t] for t in (trackers or [])], url_list=url_list or []).encode()
