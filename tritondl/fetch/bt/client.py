"""BitTorrent downloader plug-in — reference component C7
(``internal/downloader/torrent/torrent.go``).

Registration: name ``torrent``, protocol ``magnet``, extension ``.torrent``
(``torrent.go:26-36``).  ``download``: a fresh client per call rooted at the
job dir ("to prevent state leakage", ``:43``); add the magnet; wait ≤ 10 min
for metadata (``failed to get metadata``; cancellable, ``:66-76``); download
everything; report ``BytesCompleted / TotalLength * 100`` every second
(``:82-101``); wait for completion; final 100 (``:110-113``).

Fixes: ``.torrent`` URLs over http(s) — which the reference routed here by
extension and then rejected as ``unsupported scheme`` (defect B3) — are
fetched and started from their metainfo; waiting for completion honours
cancellation (B9: anacrolix ``WaitAll`` did not).
"""

from __future__ import annotations

import asyncio
import contextlib
from urllib.parse import urlparse

import aiohttp

from ...utils.log import log
from ..registry import ClientRegister, ProgressSink
from .dht import DHTNode
from .metainfo import Magnet, Metainfo, MetainfoError, parse_magnet
from .torrent import Torrent, TorrentConfig


class TorrentError(Exception):
    pass


def _parse_hostports(s: str) -> list[tuple[str, int]]:
    out = []
    for part in (s or "").split(","):
        part = part.strip()
        if not part:
            continue
        h, _, p = part.rpartition(":")
        if h.startswith("[") and h.endswith("]"):
            h = h[1:-1]                  # [v6 address]:port
        if h and p.isascii() and p.isdigit():
            out.append((h, int(p)))
    return out


class TorrentDownloader:
    streams_files = True          # download() accepts pick_files/on_file (per-file streamed uploads)

    def __init__(self, cfg: TorrentConfig | None = None, *, metadata_timeout: float = 600.0,
                 progress_interval: float = 1.0, use_dht: bool = True,
                 dht_bootstrap: list[tuple[str, int]] | None = None, extra_trackers: list[str] | None = None,
                 http_session: aiohttp.ClientSession | None = None, dht_ipv6: bool = False,
                 dht_timeout: float = 2.0, shared_dht: bool = True) -> None:
        self.cfg = cfg or TorrentConfig()
        self.metadata_timeout = metadata_timeout
        self.progress_interval = progress_interval
        self.use_dht = use_dht
        self.dht_bootstrap = dht_bootstrap or []
        self.dht_ipv6 = dht_ipv6          # BEP 32: a second DHT socket + table on IPv6
        self.dht_timeout = dht_timeout
        # one DHT node per worker process, kept across jobs (routing table stays warm,
        # buckets refreshed in the background): the reference's per-job anacrolix client
        # re-bootstrapped its DHT from the routers for every magnet
        self.shared_dht = shared_dht
        self._dht: DHTNode | None = None
        self._dht_boot: asyncio.Task | None = None
        self.extra_trackers = extra_trackers or []
        self._http = http_session

    @classmethod
    def from_config(cls, c, http=None) -> "TorrentDownloader":
        tc = TorrentConfig(listen_port=c.bt_listen_port, utp=c.bt_utp, pex=c.bt_pex, encryption=c.bt_encryption,
                           established_conns=c.bt_established_conns, half_open_conns=c.bt_half_open_conns,
                           verify_device={"on": "gpu", "off": "cpu"}.get(c.gpu_verify, c.gpu_verify),
                           upnp=c.bt_upnp, native_wire=c.bt_native_wire,
                           disk_reserve=c.disk_reserve_bytes,
                           listen_host6="::" if c.bt_dht_ipv6 else None)
        return cls(tc, metadata_timeout=c.metadata_timeout_s, progress_interval=c.progress_interval_s,
                   use_dht=c.bt_dht, dht_bootstrap=_parse_hostports(c.bt_bootstrap), dht_ipv6=c.bt_dht_ipv6)

    def register(self) -> ClientRegister:
        return ClientRegister(name="torrent", protocols=["magnet"], file_extensions=[".torrent"])

    async def _fetch_torrent_file(self, url: str) -> bytes:
        from ...utils import proxy as _proxy
        own = self._http is None
        s = self._http or aiohttp.ClientSession()
        try:
            # a .torrent URL is an ordinary web fetch: it honours the egress proxy
            # (HTTP_PROXY / HTTPS_PROXY / NO_PROXY) like the HTTP downloader
            try:
                kw, extra = _proxy.aiohttp_kwargs(_proxy.proxy_for(url), url.startswith("https:"))
            except (_proxy.ProxyConfigError, ValueError) as e:
                raise TorrentError(f"failed to fetch torrent file: {e}") from e
            async with s.get(url, timeout=aiohttp.ClientTimeout(total=120), headers=extra, **kw) as r:
                if r.status != 200:
                    raise TorrentError(f"failed to fetch torrent file: HTTP {r.status}")
                cap = 64 * 1024 * 1024          # v2 piece layers make big torrents large
                buf = bytearray()
                while True:
                    chunk = await r.content.read(1 << 20)   # read() returns what is buffered: loop to EOF
                    if not chunk:
                        break
                    buf += chunk
                    if len(buf) > cap:
                        raise TorrentError("torrent file too large")
                return bytes(buf)
        except aiohttp.ClientError as e:
            raise TorrentError(f"failed to fetch torrent file: {e}") from e
        finally:
            if own:
                await s.close()

    async def open(self, base_dir: str, url: str) -> tuple[Torrent, DHTNode | None]:
        u = urlparse(url)
        info = None
        trackers: list[str] = list(self.extra_trackers)
        peers: list[tuple[str, int]] = []
        name = ""
        webseeds: list[str] = []
        if u.scheme == "magnet":
            try:
                m: Magnet = parse_magnet(url)
            except MetainfoError as e:
                raise TorrentError(f"failed to add torrent: {e}") from e
            ih, trackers, peers, name = m.infohash, trackers + m.trackers, m.peers, m.display_name
            webseeds = list(m.web_seeds)
        elif u.scheme in ("http", "https"):
            try:
                mi = Metainfo.parse(await self._fetch_torrent_file(url))
            except MetainfoError as e:
                raise TorrentError(f"failed to add torrent: {e}") from e
            ih, info = mi.infohash, mi.info
            trackers += [t for tier in mi.announce for t in tier]
            webseeds = list(mi.url_list)
        else:
            raise TorrentError(f"unsupported scheme '{u.scheme}'")
        dht = await self._dht_node() if self.use_dht else None
        t = Torrent(ih, base_dir, self.cfg, info=info, trackers=trackers, peers=peers, dht=dht, name_hint=name,
                    webseeds=webseeds)
        await t.start()
        return t, dht

    async def _dht_node(self) -> DHTNode:
        if self.shared_dht and self._dht is not None:
            return self._dht
        bind = "127.0.0.1" if self.cfg.listen_host == "127.0.0.1" else "0.0.0.0"
        dht = await DHTNode(host=bind, bootstrap=self.dht_bootstrap, timeout=self.dht_timeout,
                            host6=("::1" if bind == "127.0.0.1" else "::") if self.dht_ipv6 else None
                            ).start(maintain=self.shared_dht)
        boot = asyncio.ensure_future(dht.bootstrap())
        if self.shared_dht:
            self._dht, self._dht_boot = dht, boot
        return dht

    async def close(self) -> None:
        """Stop the shared DHT node (Dispatcher.stop calls this on shutdown)."""
        if self._dht_boot is not None:
            self._dht_boot.cancel()
            with contextlib.suppress(BaseException):
                await self._dht_boot
            self._dht_boot = None
        if self._dht is not None:
            self._dht.stop()
            self._dht = None

    async def download(self, base_dir: str, progress: ProgressSink, url: str, *,
                       pick_files=None, on_file=None) -> None:
        """``pick_files``/``on_file``: see :meth:`Torrent.watch_files` — the
        service uses them to start each media file's upload as soon as that
        file is whole."""
        t, dht = await self.open(base_dir, url)
        stop = asyncio.Event()
        rep: asyncio.Task | None = None
        try:
            log.info("fetching torrent metadata")
            try:
                await asyncio.wait_for(t.got_info.wait(), self.metadata_timeout)
            except asyncio.TimeoutError as e:
                raise TorrentError("failed to get metadata") from e
            log.info("fetched torrent metadata")
            if on_file is not None:
                t.watch_files(pick_files, on_file)
            await t.download_all()
            total = t.info.total_length if t.info else 0

            async def reporter() -> None:
                while not stop.is_set():
                    await asyncio.sleep(self.progress_interval)
                    progress(url, (t.bytes_completed() / total * 100) if total else 100.0)

            rep = asyncio.ensure_future(reporter())
            log.info("waiting for torrent download")
            done = asyncio.ensure_future(t.complete.wait())
            bad = asyncio.ensure_future(t.failed.wait())
            try:
                await asyncio.wait({done, bad}, return_when=asyncio.FIRST_COMPLETED)
            finally:
                for f in (done, bad):
                    f.cancel()
            if not t.complete.is_set():
                raise TorrentError(f"torrent storage failed: {t.fatal}")
            progress(url, 100)
        finally:
            stop.set()
            if rep is not None:
                rep.cancel()
                with contextlib.suppress(BaseException):
                    await rep
            await t.close()
            if dht is not None and dht is not self._dht:
                dht.stop()
