"""End-to-end worker tests: the reference's job loop
(cmd/downloader/downloader.go:103-155) against in-process fakes — HTTP and
magnet jobs, decode failures, retry / dead-letter disposition (B4 fix),
broker loss mid-job (at-least-once), concurrency, CLI + cpuprofile."""

import asyncio
import os
import signal
import subprocess
import sys
import time

from tritondl.amqp.client import Client
from tritondl.amqp.codec import Properties
from tritondl.fakes.broker import Broker
from tritondl.fakes.origin import Origin
from tritondl.fakes.s3 import FakeS3
from tritondl.fakes.swarm import HTTPTracker, Seeder, magnet_for, make_payload, torrent_for
from tritondl.fetch.bt.client import TorrentDownloader
from tritondl.fetch.bt.torrent import TorrentConfig
from tritondl.fetch.http import HTTPDownloader
from tritondl.fetch.registry import Dispatcher
from tritondl.models import Convert, Download, Media
from tritondl.s3.client import S3Client
from tritondl.s3.credentials import Static
from tritondl.s3.uploader import Uploader, object_key
from tritondl.service import Service
from tritondl.utils.backoff import ExponentialBackoff
from tritondl.utils.config import Config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(coro, timeout=90):
    return asyncio.run(asyncio.wait_for(coro, timeout))


class Env:
    async def up(self, tmp_path, http=None, **cfgkw):
        self.broker = await Broker().start()
        self.origin = await Origin().start()
        self.s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        cfg = Config()
        cfg.download_dir = str(tmp_path / "downloading")
        cfg.retry_delay_s = 0
        cfg.progress_log_interval_s = 0
        cfg.heartbeat_s = 0
        for k, v in cfgkw.items():
            setattr(cfg, k, v)
        self.cfg = cfg
        http = http or HTTPDownloader(progress_interval=0.05, max_retries=1)
        bt = TorrentDownloader(TorrentConfig(listen_host="127.0.0.1", tracker_min_interval=0.5,
                                             verify_device="cpu"), progress_interval=0.05, use_dht=False)
        self.svc = Service(cfg, amqp=Client(self.broker.url, heartbeat=0, retry_delay=0,
                                            backoff=ExponentialBackoff(initial=0.02, max_interval=0.1)),
                           dispatcher=Dispatcher(cfg.download_dir, [bt, http], 0),
                           uploader=Uploader(cfg.bucket, S3Client(self.s3.endpoint, Static("ak", "sk"))))
        await self.svc.start()
        return self

    def submit(self, media: Media, headers=None, i=0, raw: bytes | None = None):
        body = raw if raw is not None else Download(created_at="t", media=media).encode()
        self.broker.inject("v1.download", f"v1.download-{i % 2}", body,
                           Properties(delivery_mode=2, headers=headers))

    async def wait_results(self, n, timeout=30):
        t0 = time.monotonic()
        while len(self.svc.results) < n:
            assert time.monotonic() - t0 < timeout, f"{len(self.svc.results)}/{n} results"
            await asyncio.sleep(0.02)
        return self.svc.results

    def converts(self):
        return [Convert.decode(m.body) for q in ("v1.convert-0", "v1.convert-1")
                for m in list(self.broker.queues.get(q).messages if q in self.broker.queues else [])]

    async def down(self):
        await self.svc.shutdown(grace=5)
        await self.s3.stop()
        await self.origin.stop()
        await self.broker.stop()


def test_http_job_end_to_end(tmp_path):
    async def main():
        e = await Env().up(tmp_path)
        data = os.urandom(2_500_000)
        url = e.origin.add("/files/The%20Movie.mkv", data)
        media = Media(id="m-1", name="The Movie", source_uri=url, type=0, status=1)
        e.submit(media)
        res = await e.wait_results(1)
        assert res[0].ok and res[0].files == 1 and res[0].bytes == len(data)
        assert e.s3.object_bytes("triton-staging", object_key("m-1", "The Movie.mkv")) == data
        await asyncio.sleep(0.05)
        conv = e.converts()
        assert len(conv) == 1 and conv[0].media_raw == media.encode()
        assert " m=+" in conv[0].created_at   # Go time.Now().String() format
        assert e.broker.queue_depth("v1.download-0") == 0 and e.broker.unacked_count() == 0
        # exchange topology for the publish side (B13)
        assert e.broker.exchanges["v1.convert"].type == "direct"
        await e.down()
    run(main())


def test_magnet_job_end_to_end(tmp_path):
    async def main():
        e = await Env().up(tmp_path)
        src = tmp_path / "seed" / "Show.S01"
        make_payload(str(src), {"season 1/ep1.mkv": 300_000, "season 1/ep2.mkv": 200_000, "info.nfo": 50,
                                "Extras/x.mkv": 10})
        info = torrent_for(str(src), 32768)
        tr = await HTTPTracker().start()
        seed = await Seeder(info, str(tmp_path / "seed"), trackers=[tr.url]).start()
        await asyncio.sleep(0.1)
        e.submit(Media(id="tv-1", source_uri=magnet_for(info, [tr.url])))
        res = await e.wait_results(1, timeout=60)
        assert res[0].ok, res[0]
        # sole TLD "Show.S01" is descended, "season 1" allowed, "Extras" pruned (process.go rules)
        keys = sorted(e.s3.buckets["triton-staging"])
        assert keys == sorted([object_key("tv-1", "ep1.mkv"), object_key("tv-1", "ep2.mkv")])
        assert res[0].files == 2
        await seed.stop()
        await tr.stop()
        await e.down()
    run(main())


def test_undecodable_body_is_nacked(tmp_path):
    async def main():
        e = await Env().up(tmp_path)
        e.submit(None, raw=b"\xff\xff\xff")
        res = await e.wait_results(1)
        assert not res[0].ok and res[0].stage == "decode"
        await asyncio.sleep(0.05)
        assert e.broker.queue_depth("v1.download-0") == 0 and e.broker.unacked_count() == 0
        assert e.broker.stats["dead"] == 1
        await e.down()
    run(main())


def test_failed_job_retried_then_dead_lettered(tmp_path):
    async def main():
        e = await Env().up(tmp_path, max_retries=2, dead_letter_topic="v1.download.dead")
        e.submit(Media(id="bad", source_uri=e.origin.url("/missing.mkv")))
        res = await e.wait_results(3)
        assert [r.ok for r in res] == [False, False, False]
        assert all(r.stage == "download" for r in res)
        await asyncio.sleep(0.1)
        dead = e.broker.drain_queue("v1.download.dead-0") + e.broker.drain_queue("v1.download.dead-1")
        assert len(dead) == 1 and dead[0].props.headers["X-Retries"] == 2
        assert dead[0].props.headers["X-Failed-Stage"] == "download"
        assert e.broker.unacked_count() == 0
        await e.down()
    run(main())


def test_unsupported_scheme_dropped_without_dlq(tmp_path):
    async def main():
        e = await Env().up(tmp_path, max_retries=0)
        e.submit(Media(id="x", source_uri="ftp://h/a.zip"))
        res = await e.wait_results(1)
        assert "unsupported fileext '.zip' or protocol 'ftp'" in res[0].error
        await asyncio.sleep(0.05)
        assert e.broker.unacked_count() == 0 and e.broker.stats["dead"] == 1
        await e.down()
    run(main())


def test_broker_drop_mid_job_redelivers(tmp_path):
    async def main():
        e = await Env().up(tmp_path)
        data = os.urandom(3_000_000)
        url = e.origin.add("/slow.mkv", data)
        e.origin.rate = 6_000_000  # ~0.5 s download
        e.submit(Media(id="slow", source_uri=url))
        await asyncio.sleep(0.2)
        await e.broker.drop_connections()
        res = await e.wait_results(2, timeout=30)
        # the in-flight job finished but its ack was lost; the redelivery completes too (at-least-once)
        assert any(r.ok for r in res)
        await asyncio.sleep(0.1)
        assert e.broker.queue_depth("v1.download-0") == 0
        assert e.s3.object_bytes("triton-staging", object_key("slow", "slow.mkv")) == data
        await e.down()
    run(main())


def test_concurrency_overlaps_jobs(tmp_path):
    async def main():
        e = await Env().up(tmp_path, concurrency=3, prefetch=3)
        e.origin.rate = 4_000_000
        for i in range(3):
            url = e.origin.add(f"/f{i}.mkv", os.urandom(1_000_000))
            e.submit(Media(id=f"c{i}", source_uri=url), i=i)
        t0 = time.monotonic()
        res = await e.wait_results(3)
        dt = time.monotonic() - t0
        assert all(r.ok for r in res)
        assert dt < 0.6, dt  # 3 x 0.25 s downloads overlapped
        await e.down()
    run(main())


def test_cli_runs_and_writes_cpuprofile(tmp_path):
    async def backends():
        b = await Broker().start()
        s = await FakeS3().start()
        return b, s

    async def main():
        b, s = await backends()
        env = dict(os.environ, RABBITMQ_ENDPOINT=b.endpoint, RABBITMQ_USERNAME="guest", RABBITMQ_PASSWORD="guest",
                   S3_ENDPOINT=s.endpoint, LOG_FORMAT="json", PYTHONPATH=ROOT)
        prof = tmp_path / "cpu.prof"
        p = await asyncio.create_subprocess_exec(sys.executable, "-m", "tritondl", "-cpuprofile", str(prof),
                                                 cwd=str(tmp_path), env=env,
                                                 stderr=asyncio.subprocess.PIPE)
        for _ in range(200):
            if "v1.download-1" in b.queues and b.queues["v1.download-1"].consumers:
                break
            await asyncio.sleep(0.05)
        assert b.queues["v1.download-1"].consumers
        p.send_signal(signal.SIGTERM)
        err = await asyncio.wait_for(p.stderr.read(), 30)
        rc = await p.wait()
        assert rc == 0, err.decode()[-2000:]
        assert b'"msg": "finished shutdown"' in err
        assert prof.exists() and prof.stat().st_size > 0
        await s.stop()
        await b.stop()
    run(main())


def test_stream_upload_overlaps_and_fails_cleanly(tmp_path):
    async def main():
        e = await Env().up(tmp_path, max_retries=0)
        data = os.urandom(6_000_000)
        url = e.origin.add("/stream.mkv", data)
        e.origin.rate = 20_000_000
        seen_put_before_done = []
        final = str(tmp_path / "downloading" / "s1" / "stream.mkv")

        class Rec(list):
            def append(self, x):
                if x[0] == "PUT" and "s1" in x[1]:
                    seen_put_before_done.append(not os.path.exists(final))
                super().append(x)
        e.s3.requests = Rec()
        e.submit(Media(id="s1", source_uri=url))
        res = await e.wait_results(1)
        assert res[0].ok and e.s3.object_bytes("triton-staging", object_key("s1", "stream.mkv")) == data
        assert seen_put_before_done == [True]   # the PUT started while the file was still .part
        # a download that dies mid-way must not leave an object behind
        url2 = e.origin.add("/dies.mkv", data)
        e.origin.cut_after, e.origin.cut_times = 1_000_000, 100
        e.submit(Media(id="s2", source_uri=url2))
        res = await e.wait_results(2, timeout=60)
        assert not res[1].ok
        assert object_key("s2", "dies.mkv") not in e.s3.buckets["triton-staging"]
        await e.down()
    run(main())
