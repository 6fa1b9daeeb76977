"""Download dispatcher + progress tracker — reference component C5
(``internal/downloader/downloader.go``).

* ``ClientImpl`` / ``ClientRegister`` / ``ProgressUpdate`` mirror
  ``downloader.go:16-61``.
* Registration fills a protocol map and a file-extension map in impl order
  (``:77-93``); the worker registers ``[torrent, http]``
  (``cmd/downloader/downloader.go:87-90``).
* ``download(id, url)``: for http/https the URL path's extension is looked
  up first, else the scheme (first registered impl wins); otherwise
  ``unsupported fileext '<ext>' or protocol '<scheme>'`` (``:138-168``).  The
  work dir ``baseDir/<id>`` (0755) is created before delegating (``:170-175``).
* Progress: impls report 0..100; the tracker drops an entry at exactly 100
  and logs ``download status`` every 5 s (``:96-130``).

Fixes: progress is guarded by the event loop (B7: the Go map was raced),
reporting after shutdown is a no-op instead of a send on a closed channel
(B9), and a media id that would escape ``baseDir`` is rejected.
"""

from __future__ import annotations

import asyncio
import math
import os
from dataclasses import dataclass, field
from typing import Protocol
from urllib.parse import urlparse

from ..utils.gocompat import go_ext, go_join
from ..utils.log import log


@dataclass
class ClientRegister:
    name: str
    protocols: list[str] = field(default_factory=list)
    file_extensions: list[str] = field(default_factory=list)


@dataclass
class ProgressUpdate:
    url: str
    progress: float  # 0..100 (B2: the reference's HTTP impl sent a 0..1 ratio)


class ProgressSink:
    """What an impl reports to (``progress chan ProgressUpdate``)."""

    def __init__(self, tracker: "ProgressTracker | None" = None) -> None:
        self.tracker = tracker

    def __call__(self, url: str, progress: float) -> None:
        if self.tracker is not None:
            self.tracker.update(ProgressUpdate(url, progress))


class ClientImpl(Protocol):
    def register(self) -> ClientRegister: ...

    async def download(self, base_dir: str, progress: ProgressSink, url: str) -> None: ...


class UnsupportedError(ValueError):
    pass


class ProgressTracker:
    def __init__(self, interval: float = 5.0) -> None:
        self.interval = interval
        self.progress: dict[str, float] = {}
        self._task: asyncio.Task | None = None
        self.closed = False
        self.history: list[ProgressUpdate] = []
        self.keep_history = False

    def update(self, p: ProgressUpdate) -> None:
        if self.closed:
            return
        if self.keep_history:
            self.history.append(p)
        if p.progress == 100:
            self.progress.pop(p.url, None)
            return
        self.progress[p.url] = p.progress

    def start(self) -> None:
        if self._task is None and self.interval > 0:
            self._task = asyncio.ensure_future(self._loop())

    async def _loop(self) -> None:
        try:
            while True:
                await asyncio.sleep(self.interval)
                for url, pct in list(self.progress.items()):
                    log.with_fields(progress=math.ceil(pct * 100) / 100, url=url).info("download status")
        except asyncio.CancelledError:
            pass

    async def stop(self) -> None:
        self.closed = True
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except asyncio.CancelledError:
                pass
            self._task = None


class Dispatcher:
    """``downloader.NewClient(ctx, baseDir, impls)``."""

    def __init__(self, base_dir: str, impls: list[ClientImpl], progress_log_interval: float = 5.0) -> None:
        if not base_dir or not os.path.isabs(base_dir):
            raise ValueError("invalid baseDir")
        self.base_dir = base_dir
        self.impls = list(impls)
        self.protocol_impl: dict[str, list[ClientImpl]] = {}
        self.file_exts_impl: dict[str, list[ClientImpl]] = {}
        self.tracker = ProgressTracker(progress_log_interval)
        self.sink = ProgressSink(self.tracker)
        for impl in impls:
            reg = impl.register()
            log.with_fields(name=reg.name, exts=reg.file_extensions, protocol=reg.protocols).info(
                "registered client implementation")
            for ext in reg.file_extensions:
                self.file_exts_impl.setdefault(ext, []).append(impl)
            for proto in reg.protocols:
                self.protocol_impl.setdefault(proto, []).append(impl)
        log.info("have %d protocol(s), and %d file extension(s) registered", len(self.protocol_impl),
                 len(self.file_exts_impl))

    def start(self) -> None:
        self.tracker.start()

    async def stop(self) -> None:
        await self.tracker.stop()
        seen = set()
        for impl in self.impls:
            close = getattr(impl, "close", None)
            if close is not None and id(impl) not in seen:
                seen.add(id(impl))
                await close()

    def select(self, url: str) -> ClientImpl:
        u = urlparse(url)
        ext = go_ext(u.path)
        log.with_fields(protocol=u.scheme, ext=ext).info("downloading file")
        impl = None
        if u.scheme in ("http", "https") and self.file_exts_impl.get(ext):
            impl = self.file_exts_impl[ext][0]
        if impl is None and self.protocol_impl.get(u.scheme):
            log.info("found supported protocol downloader")
            impl = self.protocol_impl[u.scheme][0]
        if impl is None:
            raise UnsupportedError(f"unsupported fileext '{ext}' or protocol '{u.scheme}'")
        return impl

    def job_dir(self, media_id: str) -> str:
        d = go_join(self.base_dir, media_id)
        root = go_join(self.base_dir)
        if not media_id or d == root or not d.startswith(root.rstrip("/") + "/"):
            raise ValueError(f"media id {media_id!r} escapes the download directory")
        return d

    async def download(self, media_id: str, url: str) -> str:
        impl = self.select(url)
        d = self.job_dir(media_id)
        os.makedirs(d, mode=0o755, exist_ok=True)
        await impl.download(d, self.sink, url)
        return d
