"""Spare-file recycling (tritondl/utils/spares.py): with ``cleanup`` on, a
finished job's file is renamed into the next download's ``.part`` and
overwritten instead of being deleted.  The stale bytes of the previous job
must never reach S3: every object is checked byte for byte, across smaller
and larger successors and downloads cut mid-body (resumed on the recycled
file)."""

import asyncio
import os
import random

from tritondl.amqp.client import Client
from tritondl.amqp.codec import Properties
from tritondl_testkit.fakes.broker import Broker
from tritondl_testkit.fakes.origin import Origin
from tritondl_testkit.fakes.s3 import FakeS3
from tritondl.fetch.http import HTTPDownloader
from tritondl.fetch.registry import Dispatcher
from tritondl.models import Convert, Download, Media
from tritondl.s3.client import S3Client
from tritondl.s3.credentials import Static
from tritondl.s3.uploader import Uploader, object_key
from tritondl.service import Service
from tritondl.utils import spares
from tritondl.utils.backoff import ExponentialBackoff
from tritondl.utils.config import Config


def _file(path, size, byte=b"x"):
    with open(path, "wb") as f:
        f.write(byte * size)
    return str(path)


def test_pool_bounds_and_lifo(tmp_path):
    base = tmp_path / "dl"
    base.mkdir()
    pool = spares.register(spares.SparePool(str(base), max_bytes=5 << 20, max_files=2,
                                            max_file_bytes=3 << 20, min_file_bytes=1 << 20))
    try:
        assert os.path.isdir(pool.root)
        assert not pool.offer(_file(tmp_path / "small", 1000))              # below min_file_bytes
        assert not pool.offer(_file(tmp_path / "huge", 4 << 20))            # above max_file_bytes
        assert pool.offer(_file(tmp_path / "a", 2 << 20, b"a"))
        assert pool.offer(_file(tmp_path / "b", 2 << 20, b"b"))
        assert not pool.offer(_file(tmp_path / "c", 1 << 20))               # max_files
        assert not os.path.exists(tmp_path / "b")
        job = base / "m1"
        job.mkdir()
        assert spares.pool_for(str(job)) is pool
        assert spares.pool_for(str(tmp_path / "elsewhere")) is None
        dst = str(job / "x.part")
        assert pool.take(dst)
        with open(dst, "rb") as f:
            assert f.read(1) == b"b"                 # most recent first (warmest pages)
        assert pool.take(str(job / "y.part")) and not pool.take(str(job / "z.part"))
        assert pool.taken == 2 and pool.offered == 2
        # offer_dir keeps the job dir's largest regular file
        jd = tmp_path / "done"
        (jd / "sub").mkdir(parents=True)
        _file(jd / "meta.nfo", 10)
        big = _file(jd / "sub" / "movie.mkv", 2 << 20, b"m")
        os.symlink(big, jd / "link.mkv")
        pool.offer_dir(str(jd))
        assert not os.path.exists(big) and pool.take(str(job / "w.part"))
        # release(): a download short of disk space deletes the spares first
        assert pool.offer(_file(tmp_path / "d", 2 << 20)) and pool.release() == 2 << 20
        assert os.listdir(pool.root) == [] and not pool.take(str(job / "v.part"))
    finally:
        spares.unregister(pool)
        pool.clear()
    assert spares.pool_for(str(base / "m1")) is None and not os.path.exists(pool.root)


def test_reaper_named_files_fast_path_and_fallback(tmp_path):
    """A streamed job names its one file: it is offered and the dir removed
    with one rmdir.  A dir holding anything else falls back to the walk, and
    nothing is left either way; a named file the pool refuses is deleted."""
    from tritondl.service import _Reaper
    base = tmp_path / "dl"
    base.mkdir()
    pool = spares.register(spares.SparePool(str(base), max_files=2, min_file_bytes=1 << 20))
    r = _Reaper()
    r.pool = pool
    try:
        one = base / "j1"
        one.mkdir()
        _file(one / "a.mkv", 2 << 20)
        r.submit(str(one), ["a.mkv"])
        two = base / "j2"
        (two / "extra").mkdir(parents=True)
        _file(two / "b.mkv", 2 << 20)
        _file(two / "extra" / "c.nfo", 10)
        r.submit(str(two), ["b.mkv"])
        three = base / "j3"
        three.mkdir()
        _file(three / "small.mkv", 1000)                 # below min_file_bytes: deleted, not kept
        r.submit(str(three), ["small.mkv"])
        assert r.drain(10)
        assert not one.exists() and not two.exists() and not three.exists()
        assert pool.offered == 2 and len(os.listdir(pool.root)) == 2
    finally:
        spares.unregister(pool)
        pool.clear()


def test_stale_pools_of_dead_processes(tmp_path):
    mine = tmp_path / f"{spares.PREFIX}{os.getpid()}"
    mine.mkdir()
    dead = tmp_path / f"{spares.PREFIX}999999999"
    dead.mkdir()
    (tmp_path / f"{spares.PREFIX}junk").mkdir()
    (tmp_path / "job").mkdir()
    assert spares.stale_pools(str(tmp_path)) == [str(dead)]


def test_recycled_files_never_leak_previous_bytes(tmp_path):
    rng = random.Random(5)
    mib = 1 << 20
    # alternate bigger and smaller successors; every job's bytes are distinct
    sizes = [3 * mib, 2 * mib, 5 * mib, 1 * mib + 123, 4 * mib + 7, 2 * mib - 1, 6 * mib, 3 * mib + 5,
             2 * mib, 5 * mib + 11, 1 * mib, 4 * mib]
    payloads = [rng.randbytes(n) for n in sizes]

    async def main():
        broker = await Broker().start()
        origin = await Origin().start()
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        cfg = Config()
        cfg.download_dir = str(tmp_path / "dl")
        cfg.retry_delay_s = 0
        cfg.max_retries = 10
        cfg.concurrency = 2
        cfg.prefetch = 2
        cfg.progress_log_interval_s = 0
        cfg.heartbeat_s = 0
        cfg.cleanup = True
        http = HTTPDownloader(progress_interval=0.05, max_retries=3)
        svc = Service(cfg, amqp=Client(broker.url, prefetch=2, heartbeat=0, retry_delay=0,
                                       backoff=ExponentialBackoff(initial=0.01, max_interval=0.05)),
                      dispatcher=Dispatcher(cfg.download_dir, [http], 0),
                      uploader=Uploader(cfg.bucket, S3Client(s3.endpoint, Static("ak", "sk"), max_retries=2,
                                                             part_size=5 << 20, multipart_threshold=6 << 20)))
        await svc.start()
        pool = svc._reaper.pool
        assert pool is not None and spares.pool_for(os.path.join(cfg.download_dir, "x")) is pool
        for i, data in enumerate(payloads):
            url = origin.add(f"/m/r{i}.mkv", data)
            body = Download(created_at="t", media=Media(id=f"r{i}", source_uri=url)).encode()
            broker.inject("v1.download", f"v1.download-{i % 2}", body, Properties(delivery_mode=2))
            if i in (4, 8):
                origin.cut_after, origin.cut_times = 300_000, 1       # a resumed download on a spare
        for _ in range(600):
            conv = {Convert.decode(m.body).media.id
                    for q in ("v1.convert-0", "v1.convert-1") if q in broker.queues
                    for m in list(broker.queues[q].messages)}
            if len(conv) == len(payloads) and broker.unacked_count() == 0:
                break
            await asyncio.sleep(0.05)
        taken = pool.taken
        await svc.shutdown(grace=5)
        got = {i: s3.object_bytes("triton-staging", object_key(f"r{i}", f"r{i}.mkv")) for i in range(len(payloads))}
        await s3.stop()
        await origin.stop()
        await broker.stop()
        for i, data in enumerate(payloads):
            assert len(got[i]) == len(data) and got[i] == data, i
        assert taken >= 3, taken                      # the recycling path actually ran
        assert not [n for n in os.listdir(cfg.download_dir) if n.startswith(spares.PREFIX)]
        assert spares.pool_for(os.path.join(cfg.download_dir, "x")) is None
    asyncio.run(asyncio.wait_for(main(), 120))


def test_download_short_of_space_deletes_spares_first(tmp_path, monkeypatch):
    import tritondl.fetch.http as fh
    from tritondl.utils.disk import DiskSpaceError

    base = tmp_path / "dl"
    (base / "job").mkdir(parents=True)
    pool = spares.register(spares.SparePool(str(base)))
    checks = []

    def check_space(path, need, reserve=0):
        checks.append(len(pool._files))
        if pool._files:                    # the spares are what fills the disk
            raise DiskSpaceError("no space")
    monkeypatch.setattr(fh, "check_space", check_space)
    data = random.Random(1).randbytes(3 << 20)

    async def main():
        origin = await Origin().start()
        try:
            url = origin.add("/m/a.mkv", data)
            assert pool.offer(_file(tmp_path / "old", 2 << 20, b"o"))
            await HTTPDownloader(progress_interval=0.05).download(str(base / "job"), lambda *a: None, url)
        finally:
            await origin.stop()
    try:
        asyncio.run(asyncio.wait_for(main(), 60))
        with open(base / "job" / "a.mkv", "rb") as f:
            assert f.read() == data
        assert checks == [1, 0] and pool.taken == 0 and os.listdir(pool.root) == []
    finally:
        spares.unregister(pool)
        pool.clear()

