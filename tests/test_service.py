"""End-to-end worker tests: the reference's job loop
(cmd/downloader/downloader.go:103-155) against in-process fakes — HTTP and
magnet jobs, decode failures, retry / dead-letter disposition (B4 fix),
broker loss mid-job (at-least-once), concurrency, CLI + cpuprofile."""

import asyncio
import os
import shutil
import signal
import subprocess
import sys
import time

import pytest

from tritondl.amqp.client import Client
from tritondl.amqp.codec import Properties
from tritondl_testkit.fakes.broker import Broker
from tritondl_testkit.fakes.origin import Origin
from tritondl_testkit.fakes.s3 import FakeS3
from tritondl_testkit.fakes.swarm import HTTPTracker, Seeder, magnet_for, make_payload, torrent_for
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


def _dlq(broker, topic="v1.download.dead"):
    return broker.drain_queue(f"{topic}-0") + broker.drain_queue(f"{topic}-1")


def test_undecodable_body_is_dead_lettered(tmp_path):
    async def main():
        e = await Env().up(tmp_path)
        e.submit(None, raw=b"\xff\xff\xff")
        res = await e.wait_results(1)
        assert not res[0].ok and res[0].stage == "decode"
        await asyncio.sleep(0.05)
        assert e.broker.queue_depth("v1.download-0") == 0 and e.broker.unacked_count() == 0
        dead = _dlq(e.broker)
        assert len(dead) == 1 and dead[0].body == b"\xff\xff\xff"
        assert dead[0].props.headers["X-Failed-Stage"] == "decode"
        await e.down()
    run(main())


def test_drop_failed_opt_out_nacks(tmp_path):
    async def main():
        e = await Env().up(tmp_path, max_retries=0, drop_failed=True)
        e.submit(None, raw=b"\xff\xff\xff")
        e.submit(Media(id="x", source_uri="ftp://h/a.zip"), i=1)
        await e.wait_results(2)
        await asyncio.sleep(0.05)
        assert e.broker.unacked_count() == 0 and e.broker.stats["dead"] == 2
        assert _dlq(e.broker) == []
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


def test_failed_retry_publish_still_settles_the_delivery(tmp_path, monkeypatch):
    """A retry whose publish fails falls back to the dead-letter queue; if
    that publish fails too, the delivery is parked (re-published to its own
    queue with X-Retries+1 after ``retry_delay_max_s``), never nack-requeued.
    Either way the prefetch-1 slot is freed, so the consumer never stalls."""
    from tritondl.amqp import client as amqp_client

    async def no_retry(self, delay=None):
        raise RuntimeError("PRECONDITION_FAILED - inequivalent arg 'x-message-ttl'")
    monkeypatch.setattr(amqp_client.Delivery, "retry", no_retry)
    real_publish = amqp_client.Client.publish
    fails = {"n": 1}

    async def flaky_publish(self, topic, body, *a, **kw):
        if topic.endswith(".dead") and fails["n"]:
            fails["n"] -= 1
            raise RuntimeError("publish nacked")
        return await real_publish(self, topic, body, *a, **kw)
    monkeypatch.setattr(amqp_client.Client, "publish", flaky_publish)

    async def main():
        e = await Env().up(tmp_path, max_retries=3, retry_delay_max_s=0.05)
        e.submit(Media(id="x", source_uri="ftp://h/a.zip"))
        res = await e.wait_results(2)               # parked once, handled again
        assert [r.ok for r in res] == [False, False]
        await asyncio.sleep(0.05)
        dead = _dlq(e.broker)
        assert len(dead) == 1 and e.broker.unacked_count() == 0
        assert dead[0].props.headers["X-Retries"] == 1
        assert e.svc.metrics.get("jobs_parked") == 1 and e.broker.stats["requeued"] == 0
        e.submit(Media(id="y", source_uri="ftp://h/b.zip"))   # the consumer still takes jobs
        await e.wait_results(3)
        await e.down()
    run(main())


def test_unsupported_scheme_dead_lettered(tmp_path):
    async def main():
        e = await Env().up(tmp_path, max_retries=0)
        e.submit(Media(id="x", source_uri="ftp://h/a.zip"))
        res = await e.wait_results(1)
        assert "unsupported fileext '.zip' or protocol 'ftp'" in res[0].error
        await asyncio.sleep(0.05)
        assert e.broker.unacked_count() == 0
        dead = _dlq(e.broker)
        assert len(dead) == 1 and "unsupported fileext" in dead[0].props.headers["X-Error"]
        assert dead[0].props.headers["X-Original-Routing-Key"] == "v1.download-0"
        await e.down()
    run(main())


def test_s3_outage_longer_than_retry_budget_loses_no_job(tmp_path):
    """Every retry waits in a broker delay queue (x-message-ttl + DLX back to
    the shard); once the budget is spent the job lands in the dead-letter
    queue.  An outage outlasting the whole budget must leave every job in the
    DLQ — none dropped, none stuck unacked."""
    async def main():
        e = await Env().up(tmp_path, max_retries=3, retry_delay_s=0.05, retry_backoff=2.0)
        e.svc.uploader.client.max_retries = 0
        e.s3.fail_for(60.0)
        n = 6
        for k in range(n):
            url = e.origin.add(f"/o{k}.mkv", os.urandom(20_000))
            e.submit(Media(id=f"o{k}", source_uri=url), i=k)
        await e.wait_results(n * 4, timeout=60)          # 1 try + 3 retries each
        await asyncio.sleep(0.2)
        dead = _dlq(e.broker)
        assert sorted(Download.decode(m.body).media.id for m in dead) == [f"o{k}" for k in range(n)]
        assert all(m.props.headers["X-Retries"] == 3 and m.props.headers["X-Failed-Stage"] == "upload"
                   for m in dead)
        assert e.broker.unacked_count() == 0
        assert all(len(q.messages) == 0 for name, q in e.broker.queues.items() if not name.startswith("v1.convert"))
        # the delays grew per retry: 50, 100, 200 ms queues were used
        delay_qs = sorted(q for q in e.broker.queues if ".retry." in q)
        assert {q.split(".retry.")[1] for q in delay_qs} == {"50ms", "100ms", "200ms"}
        assert e.broker.stats["expired"] == n * 3
        assert e.converts() == []
        await e.down()
    run(main())


def test_failing_job_does_not_hold_the_slot(tmp_path):
    """The reference's Error() slept 10 s in the job goroutine; here the delay
    lives in the broker, so the next job starts at once."""
    async def main():
        e = await Env().up(tmp_path, max_retries=5, retry_delay_s=5.0)
        e.submit(Media(id="bad", source_uri=e.origin.url("/missing.mkv")))
        await e.wait_results(1)
        t0 = time.monotonic()
        good = e.origin.add("/ok.mkv", os.urandom(50_000))
        e.submit(Media(id="good", source_uri=good), i=1)
        res = await e.wait_results(2, timeout=10)
        assert res[1].ok and time.monotonic() - t0 < 2.0
        assert e.broker.queue_depth("v1.download-0.retry.5000ms") == 1
        held = e.broker.queues["v1.download-0.retry.5000ms"].messages[0]
        assert held.props.headers["X-Retries"] == 1
        for _ in range(100):            # the result is recorded before the (pipelined) ack lands
            if e.broker.unacked_count() == 0:
                break
            await asyncio.sleep(0.02)
        assert e.broker.unacked_count() == 0
        await e.down()
    run(main())


def test_empty_s3_endpoint_is_fatal_before_consuming(tmp_path):
    """Reference: NewUploader error → log.Fatal before the job loop
    (downloader.go:95-98).  The worker must exit non-zero without taking a job."""
    async def main():
        b = await Broker().start()
        b.inject("", "nothing", b"")        # no-op; the broker has no queues yet
        env = dict(os.environ, RABBITMQ_ENDPOINT=b.endpoint, RABBITMQ_USERNAME="guest", RABBITMQ_PASSWORD="guest",
                   S3_ENDPOINT="", TRITONDL_DOWNLOAD_DIR=str(tmp_path / "dl"), TRITONDL_GPU_VERIFY="off")
        p = await asyncio.create_subprocess_exec(sys.executable, "-m", "tritondl", cwd=ROOT, env=env,
                                                 stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.STDOUT)
        out, _ = await asyncio.wait_for(p.communicate(), 60)
        assert p.returncode != 0, out.decode()
        assert b"S3_ENDPOINT" in out
        assert b.stats["published"] == 0 and not b.conns and "v1.download-0" not in b.queues
        await b.stop()
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


def test_same_job_twice_runs_one_at_a_time(tmp_path):
    """Two deliveries of one media id at once (a redelivery while the first
    still runs): the second waits for the first instead of truncating the
    file it is uploading from, then finds it complete and re-uploads it."""
    import fcntl

    async def main():
        e = await Env().up(tmp_path, concurrency=2, prefetch=2)
        e.origin.rate = 4_000_000
        data = os.urandom(1_000_000)
        url = e.origin.add("/same.mkv", data)
        e.submit(Media(id="dup", source_uri=url), i=0)
        e.submit(Media(id="dup", source_uri=url), i=1)
        res = await e.wait_results(2)
        assert all(r.ok for r in res), res
        assert e.s3.object_bytes("triton-staging", object_key("dup", "same.mkv")) == data
        assert [m[0] for m in e.origin.requests].count("GET") == 2   # the second one: probe, file complete
        # another worker process holding the job dir's lock blocks a delivery until released
        d = tmp_path / "downloading" / "held"
        d.mkdir(parents=True)
        fd = os.open(d, os.O_RDONLY | os.O_DIRECTORY)
        fcntl.flock(fd, fcntl.LOCK_EX)
        url2 = e.origin.add("/held.mkv", b"h" * 1000)
        e.submit(Media(id="held", source_uri=url2), i=0)
        await asyncio.sleep(0.3)
        assert len(e.svc.results) == 2                                # still waiting on the lock
        os.close(fd)
        res = await e.wait_results(3)
        assert res[-1].ok
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


def test_streamed_job_starts_the_download_pump_before_the_upload(tmp_path, monkeypatch):
    """The single-stream fetch runs inline in the downloader's task, which is
    made before the upload's, so the receive pump starts ahead of the PUT's
    SigV4 setup (profiles/r05_gil_ab/: +8 % on the headline job)."""
    from tritondl.utils import rawhttp
    if rawhttp.relay_module() is None:
        pytest.skip("native relay not built")
    events: list = []
    monkeypatch.setattr(rawhttp, "TRACE", events)

    async def main():
        e = await Env().up(tmp_path)
        for k in range(3):
            e.submit(Media(id=f"o{k}", source_uri=e.origin.add(f"/o{k}.mkv", os.urandom(2_000_000))))
        res = await e.wait_results(3)
        assert all(r.ok for r in res), res
        await e.down()
    run(main())
    names = [n for n, _t in events]
    starts = [i for i, n in enumerate(names) if n == "job_start"] + [len(names)]
    for a, b in zip(starts, starts[1:]):
        job = names[a:b]
        assert job.index("get_pump_start") < job.index("put_pump_start"), job


def test_magnet_job_streams_each_file_as_it_completes(tmp_path):
    """Torrent jobs upload every selected file as soon as its last piece is
    verified (files fetched in order), not after the whole torrent: the first
    file's upload starts while most of the swarm download is still ahead."""
    async def main():
        e = await Env().up(tmp_path)
        src = tmp_path / "seed" / "Show.S02"
        sizes = {"season 2/e1.mkv": 2_000_000, "season 2/e2.mkv": 2_000_000, "season 2/e3.mkv": 8_000_000,
                 "notes.txt": 1000}
        make_payload(str(src), sizes)
        info = torrent_for(str(src), 32768)
        tr = await HTTPTracker().start()
        seed = await Seeder(info, str(tmp_path / "seed"), trackers=[tr.url]).start()
        e.submit(Media(id="tv-2", source_uri=magnet_for(info, [tr.url])))
        res = await e.wait_results(1, timeout=60)
        assert res[0].ok, res[0]
        m = res[0].marks
        # the first file (2 of 12 MB, fetched first) completed and its upload started while
        # the swarm was still downloading the rest: well before the download finished
        assert m["first_file"] < 0.8 * m["fetched"] and m["first_file"] < m["first_upload"], m
        keys = sorted(e.s3.buckets["triton-staging"])
        assert keys == sorted(object_key("tv-2", f"e{k}.mkv") for k in (1, 2, 3))
        for k in (1, 2, 3):
            assert e.s3.object_bytes("triton-staging", object_key("tv-2", f"e{k}.mkv")) == \
                (src / "season 2" / f"e{k}.mkv").read_bytes()
        assert res[0].files == 3 and res[0].bytes == 12_000_000
        await seed.stop()
        await tr.stop()
        await e.down()
    run(main())


def test_magnet_job_streamed_upload_failure_fails_job(tmp_path):
    """An S3 failure of a streamed torrent file upload cancels the swarm
    download and fails the job at stage ``upload`` (then dead-letters it)."""
    async def main():
        e = await Env().up(tmp_path, max_retries=0)
        e.svc.uploader.client.max_retries = 0
        src = tmp_path / "seed" / "Film"
        make_payload(str(src), {"a.mkv": 1_500_000, "b.mkv": 1_500_000})
        info = torrent_for(str(src), 32768)
        tr = await HTTPTracker().start()
        seed = await Seeder(info, str(tmp_path / "seed"), trackers=[tr.url]).start()
        e.s3.create_bucket("triton-staging")
        e.s3.fail_for(30.0)
        e.submit(Media(id="f-1", source_uri=magnet_for(info, [tr.url])))
        res = await e.wait_results(1, timeout=60)
        assert not res[0].ok and res[0].stage == "upload", res[0]
        await asyncio.sleep(0.1)
        dead = _dlq(e.broker)
        assert len(dead) == 1 and dead[0].props.headers["X-Failed-Stage"] == "upload"
        await seed.stop()
        await tr.stop()
        await e.down()
    run(main())


def test_failed_multipart_upload_resumes_on_retry(tmp_path):
    """An S3 failure mid multipart upload fails the job; the retry (broker
    delay queue) finds the file already downloaded and continues the kept
    upload: parts that landed are not sent again."""
    async def main():
        e = await Env().up(tmp_path, max_retries=2)
        c = e.svc.uploader.client
        c.part_size, c.multipart_threshold, c.parallel_parts, c.max_retries = 5 << 20, 5 << 20, 1, 0
        e.s3.store = "memory"
        data = os.urandom((16 << 20) + 77)
        url = e.origin.add("/season/pack.mkv", data)
        e.s3.fail_parts, e.s3.fail_parts_once = {3}, True   # once: the retry may start before we look
        e.submit(Media(id="mp-1", source_uri=url))
        res = await e.wait_results(2, timeout=60)
        assert not res[0].ok and res[0].stage == "upload"
        assert res[1].ok, res[1]
        parts = [int(r[1].split("partNumber=")[1].split("&")[0]) for r in e.s3.requests
                 if r[0] == "PUT" and "partNumber=" in r[1]]
        assert parts == [1, 2, 3, 3, 4], parts          # 1st try: 1, 2, (3 failed); retry: 3, 4
        assert e.s3.object_bytes("triton-staging", object_key("mp-1", "pack.mkv")) == data
        await e.down()
    run(main())


def test_wait_finished_wakes_on_result_and_times_out():
    """Service.wait_finished is woken by the recorded result itself (the
    bench harness waits on it instead of polling the workers' loop); the
    count keeps growing when the recent-results list is trimmed."""
    from tritondl.service import JobResult

    async def main():
        svc = Service(Config(bucket="b", s3_endpoint="http://127.0.0.1:1"))
        w = asyncio.ensure_future(svc.wait_finished(2, timeout=5))
        await asyncio.sleep(0)
        svc._record(JobResult(True, "done"))
        await asyncio.sleep(0)
        assert not w.done()
        svc._record(JobResult(True, "done"))
        await asyncio.wait_for(w, 1)
        assert svc.jobs_finished == 2 and not svc._finish_waiters
        await svc.wait_finished(1)                     # already reached: returns at once
        for _ in range(10001):
            svc._record(JobResult(True, "done"))
        assert len(svc.results) < svc.jobs_finished == 10003
        try:
            await svc.wait_finished(10004, timeout=0.05)
        except TimeoutError as e:
            assert "10003/10004" in str(e)
        else:
            raise AssertionError("no timeout")
        assert not svc._finish_waiters

    asyncio.run(main())


def _hold_lock_proc(path):
    """A separate process holding the job dir's flock (another worker mid-job)."""
    code = ("import fcntl, os, sys, time\n"
            "fd = os.open(sys.argv[1], os.O_RDONLY | os.O_DIRECTORY)\n"
            "fcntl.flock(fd, fcntl.LOCK_EX)\n"
            "print('locked', flush=True)\n"
            "time.sleep(120)\n")
    p = subprocess.Popen([sys.executable, "-c", code, str(path)], stdout=subprocess.PIPE)
    assert p.stdout.readline().strip() == b"locked"
    return p


def test_sigterm_while_waiting_on_a_job_lock_exits_promptly(tmp_path):
    """VERDICT r03 Weak #3: a delivery waiting on another process's job-dir
    lock must not pin the worker past SIGTERM (the old wait was a blocking
    flock in an executor thread that the interpreter joined at exit)."""
    async def main():
        b = await Broker().start()
        s = await FakeS3().start()
        o = await Origin().start()
        dl = tmp_path / "downloading"
        (dl / "held").mkdir(parents=True)
        holder = _hold_lock_proc(dl / "held")
        env = dict(os.environ, RABBITMQ_ENDPOINT=b.endpoint, RABBITMQ_USERNAME="guest", RABBITMQ_PASSWORD="guest",
                   S3_ENDPOINT=s.endpoint, LOG_FORMAT="json", PYTHONPATH=ROOT, TRITONDL_DOWNLOAD_DIR=str(dl),
                   TRITONDL_GPU_VERIFY="off", TRITONDL_RETRY_DELAY="5")
        p = await asyncio.create_subprocess_exec(sys.executable, "-m", "tritondl", cwd=str(tmp_path), env=env,
                                                 stderr=asyncio.subprocess.PIPE)
        try:
            for _ in range(400):
                if "v1.download-1" in b.queues and b.queues["v1.download-1"].consumers:
                    break
                await asyncio.sleep(0.05)
            url = o.add("/held.mkv", b"h" * 1000)
            b.inject("v1.download", "v1.download-0", Download(created_at="t", media=Media(id="held", source_uri=url))
                     .encode(), Properties(delivery_mode=2))
            err = b""
            while b"waiting for it" not in err:
                err += await asyncio.wait_for(p.stderr.readline(), 20)
            t0 = time.monotonic()
            p.send_signal(signal.SIGTERM)
            err += await asyncio.wait_for(p.stderr.read(), 20)
            rc = await p.wait()
            assert rc == 0, err.decode()[-2000:]
            assert time.monotonic() - t0 < 5.0
            assert b"handing the delivery back" in err
            # the job went back to the broker (delay queue), unspent: nothing lost, nothing stuck
            held = b.queues["v1.download-0.retry.5000ms"].messages
            assert len(held) == 1 and held[0].props.headers["X-Retries"] == 0
        finally:
            holder.kill()
            holder.wait()
            if p.returncode is None:
                p.kill()
                await p.wait()
        await o.stop()
        await s.stop()
        await b.stop()
    run(main())


def test_job_lock_held_too_long_hands_the_delivery_back(tmp_path):
    async def main():
        e = await Env().up(tmp_path, job_lock_wait_s=0.3, retry_delay_s=0.2)
        d = tmp_path / "downloading" / "busy"
        d.mkdir(parents=True)
        holder = _hold_lock_proc(d)
        try:
            url = e.origin.add("/busy.mkv", b"b" * 5000)
            e.submit(Media(id="busy", source_uri=url))
            res = await e.wait_results(1)
            assert res[0].stage == "lock" and e.svc.metrics.get("jobs", status="busy") == 1
            # the slot is free while it waits in the broker
            url2 = e.origin.add("/other.mkv", b"o" * 5000)
            e.submit(Media(id="other", source_uri=url2), i=1)
            res = await e.wait_results(2)
            assert res[1].ok
        finally:
            holder.kill()
            holder.wait()
        res = await e.wait_results(3)                  # back from the delay queue, lock free now
        assert res[2].ok
        assert e.s3.object_bytes("triton-staging", object_key("busy", "busy.mkv")) == b"b" * 5000
        await e.down()
    run(main())


def test_cleanup_redelivery_waiting_on_the_lock_gets_a_live_dir(tmp_path):
    """with cleanup on, the first delivery renames its job dir away
    when it finishes; a second delivery that was waiting on the lock must not
    end up locking (and writing into) the renamed inode."""
    async def main():
        e1 = await Env().up(tmp_path, cleanup=True, recycle_bytes=0)
        cfg2 = Config()
        for k, v in vars(e1.cfg).items():
            setattr(cfg2, k, v)
        svc2 = Service(cfg2, amqp=Client(e1.broker.url, heartbeat=0, retry_delay=0),
                       dispatcher=Dispatcher(cfg2.download_dir, [HTTPDownloader(progress_interval=0.05,
                                                                                max_retries=1)], 0),
                       uploader=Uploader(cfg2.bucket, S3Client(e1.s3.endpoint, Static("ak", "sk"))))
        await svc2.start()
        e1.origin.rate = 3_000_000
        data = os.urandom(900_000)
        url = e1.origin.add("/twice.mkv", data)
        e1.submit(Media(id="twice", source_uri=url), i=0)
        e1.submit(Media(id="twice", source_uri=url), i=0)     # round-robin: the other service's consumer
        await asyncio.sleep(0.05)
        assert e1.broker.queues["v1.download-0"].delivered_total == 2
        t0 = time.monotonic()
        while len(e1.svc.results) + len(svc2.results) < 2:
            assert time.monotonic() - t0 < 30
            await asyncio.sleep(0.02)
        res = e1.svc.results + svc2.results
        assert all(r.ok for r in res), res
        assert len(e1.svc.results) == 1 and len(svc2.results) == 1      # one each: the flock path
        assert e1.s3.object_bytes("triton-staging", object_key("twice", "twice.mkv")) == data
        await svc2.shutdown(grace=5)
        await e1.down()
    run(main())


def test_pipelined_commit_overlaps_confirms_but_acks_after_them(tmp_path):
    """A job frees its loop once its upload is done: its publish confirm and
    ack overlap the next job.  Every ack still follows its own confirmed
    v1.convert publish (at-least-once), and the reference's one-job-at-a-time
    data path is kept (concurrency 1)."""
    async def main():
        e = await Env().up(tmp_path, pipeline_commit=True, pipeline_commit_min_ms=0)
        e.broker.confirm_delay = 0.25
        for k in range(4):
            url = e.origin.add(f"/p{k}.mkv", os.urandom(50_000))
            e.submit(Media(id=f"p{k}", source_uri=url), i=k)
        t0 = time.monotonic()
        res = await e.wait_results(4, timeout=20)
        dt = time.monotonic() - t0
        assert all(r.ok for r in res)
        assert dt < 0.8, dt                      # serial commits would take >= 4 x 0.25 s
        for _ in range(200):                     # the last ack frame may still be on its way
            if sum(1 for x in e.broker.events if x[0] == "ack") == 4:
                break
            await asyncio.sleep(0.01)
        ev = [x for x in e.broker.events if x[0] == "ack" or x[1] == "v1.convert"]
        # the k-th ack comes after the k-th convert publish's confirm
        confs = [i for i, x in enumerate(ev) if x[0] == "confirm"]
        acks = [i for i, x in enumerate(ev) if x[0] == "ack"]
        assert len(confs) == len(acks) == 4 and all(a > c for c, a in zip(confs, acks)), ev
        await e.down()
    run(main())


def test_pipelined_commit_off_is_serial(tmp_path):
    async def main():
        e = await Env().up(tmp_path, pipeline_commit=False)
        e.broker.confirm_delay = 0.2
        for k in range(3):
            url = e.origin.add(f"/s{k}.mkv", os.urandom(20_000))
            e.submit(Media(id=f"s{k}", source_uri=url), i=k)
        t0 = time.monotonic()
        await e.wait_results(3, timeout=20)
        assert time.monotonic() - t0 >= 0.6
        await e.down()
    run(main())


def test_heap_trim_runs_periodically(tmp_path):
    """glibc arenas' free memory is handed back on a timer (RSS stays flat
    over a long run, profiles/r04_soak60/)."""
    from tritondl.service import _malloc_trim

    async def main():
        e = await Env().up(tmp_path, malloc_trim_s=0.1)
        await asyncio.sleep(0.5)
        if _malloc_trim() is not None:
            assert e.svc._trimmer is not None and not e.svc._trimmer.done()
        await e.down()
        assert e.svc._trimmer is None or e.svc._trimmer.done()
    run(main())


def test_malloc_policy_keeps_big_blocks_out_of_the_arenas():
    """tune_malloc pins glibc's mmap threshold: after a 4 MiB block is freed
    (which, left dynamic, raises the threshold to 4 MiB) a 1 MiB block is
    still mmapped rather than carved from an arena.  Run in a child so this
    process's heap policy is untouched."""
    import subprocess
    import sys
    code = r"""
import ctypes, sys
from tritondl.service import tune_malloc
libc = ctypes.CDLL("libc.so.6")
libc.malloc.restype = ctypes.c_void_p
libc.malloc.argtypes = [ctypes.c_size_t]
libc.free.argtypes = [ctypes.c_void_p]
class MI2(ctypes.Structure):
    _fields_ = [(n, ctypes.c_size_t) for n in ("arena", "ordblks", "smblks", "hblks", "hblkhd", "usmblks",
                                               "fsmblks", "uordblks", "fordblks", "keepcost")]
libc.mallinfo2.restype = MI2
fixed = sys.argv[1] == "fixed"
applied = tune_malloc(262144 if fixed else 0)
libc.free(libc.malloc(4 << 20))
before = libc.mallinfo2().hblks
q = libc.malloc(1 << 20)
print(applied, libc.mallinfo2().hblks - before)
libc.free(q)
"""
    out = {}
    for arm in ("fixed", "dynamic"):
        p = subprocess.run([sys.executable, "-c", code, arm], capture_output=True, text=True, timeout=60,
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert p.returncode == 0, p.stderr
        out[arm] = p.stdout.split()[-1]
        if arm == "fixed":
            assert "262144" in p.stdout
    assert out == {"fixed": "1", "dynamic": "0"}


def test_malloc_policy_trim_threshold_stops_medium_block_thrash():
    """With the mmap threshold pinned, glibc's trim threshold stays at 128 KiB
    and a 200 KiB malloc/free loop gives its pages back and faults them in on
    every cycle; the worker's default trim threshold (4 MiB) stops that."""
    import subprocess
    import sys
    code = r"""
import ctypes, resource, sys
from tritondl.service import tune_malloc
libc = ctypes.CDLL("libc.so.6")
libc.malloc.restype = ctypes.c_void_p
libc.malloc.argtypes = [ctypes.c_size_t]
libc.free.argtypes = [ctypes.c_void_p]
libc.memset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
import threading
tune_malloc(262144, trim_threshold=int(sys.argv[1]))
out = []
def loop():
    # on a fresh thread: its own arena has no free holes left by imports, so each
    # block comes from the arena's top (the main heap's layout shifts with every import)
    r0 = resource.getrusage(resource.RUSAGE_THREAD).ru_minflt
    for _ in range(2000):
        p = libc.malloc(200 << 10)
        libc.memset(p, 1, 200 << 10)
        libc.free(p)
    out.append(resource.getrusage(resource.RUSAGE_THREAD).ru_minflt - r0)
t = threading.Thread(target=loop)
t.start()
t.join()
print(out[0])
"""
    from tritondl.utils.config import Config
    faults = {}
    for trim in (128 << 10, Config().malloc_trim_threshold):     # glibc's 128 KiB set explicitly
        p = subprocess.run([sys.executable, "-c", code, str(trim)], capture_output=True, text=True, timeout=60,
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert p.returncode == 0, p.stderr
        faults[trim] = int(p.stdout.split()[-1])
    assert faults[128 << 10] > 10 * 2000 and faults[4 << 20] < 2000, faults


def test_pipelined_commit_follows_the_confirm_round_trip(tmp_path):
    """Commits are pipelined only while the broker's publish -> confirm round
    trip is long enough to be worth it (on loopback the overlap cost ~4 %,
    under a 2-20 ms round trip it gained 30-47 %: profiles/r05_rtt_ab/)."""
    async def main():
        e = await Env().up(tmp_path, pipeline_commit=True, pipeline_commit_min_ms=10.0)
        for k in range(3):
            url = e.origin.add(f"/f{k}.mkv", os.urandom(20_000))
            e.submit(Media(id=f"f{k}", source_uri=url), i=k)
        await e.wait_results(3)
        assert e.svc.amqp.confirm_ewma is not None and e.svc.amqp.confirm_ewma < 0.010
        assert e.svc.metrics.get("pipeline_commit_active") == 0.0
        e.broker.confirm_delay = 0.05                    # a 50 ms confirm: pipeline
        for k in range(3, 12):
            url = e.origin.add(f"/f{k}.mkv", os.urandom(20_000))
            e.submit(Media(id=f"f{k}", source_uri=url), i=k)
        await e.wait_results(12, timeout=20)
        assert e.svc.amqp.confirm_ewma >= 0.010
        assert e.svc.metrics.get("pipeline_commit_active") == 1.0
        assert all(r.ok for r in e.svc.results)
        await e.down()
    run(main())


def test_startup_heap_is_frozen_and_the_knob_turns_it_off(monkeypatch):
    """Service.start moves the start-up heap to the permanent generation
    (a full collection over torch's ~180k objects stalls the loop 40-100 ms);
    TRITONDL_GC_FREEZE=0 leaves the collector alone."""
    import gc
    from tritondl.service import freeze_startup_heap
    from tritondl.utils.config import Config
    try:
        assert freeze_startup_heap() > 1000 and gc.get_freeze_count() > 1000
    finally:
        gc.unfreeze()
    assert Config().gc_freeze is True
    monkeypatch.setenv("TRITONDL_GC_FREEZE", "0")
    assert Config.from_env(argv=[]).gc_freeze is False


def test_dead_lettered_job_leaves_no_files_but_a_retried_one_keeps_them(tmp_path):
    """With cleanup on, a job that failed for good (dead-lettered) has its
    partial download removed, or a poison torrent's GBs would stay on disk
    forever; while retries remain, the files stay for the next attempt to
    resume from."""
    async def main():
        e = await Env().up(tmp_path, max_retries=1, retry_delay_s=0.3, cleanup=True)
        e.svc.uploader.client.max_retries = 0
        e.s3.fail_for(60.0)
        url = e.origin.add("/keep.mkv", os.urandom(200_000))
        e.submit(Media(id="pz", source_uri=url))
        await e.wait_results(1, timeout=30)
        job_dir = os.path.join(e.cfg.download_dir, "pz")
        assert os.path.exists(os.path.join(job_dir, "keep.mkv"))        # retry pending: kept
        await e.wait_results(2, timeout=30)
        for _ in range(100):
            if not os.path.exists(job_dir) and not any(".deleting-" in n for n in os.listdir(e.cfg.download_dir)):
                break
            await asyncio.sleep(0.02)
        assert len(_dlq(e.broker)) == 1
        assert not os.path.exists(job_dir)
        assert not any(".deleting-" in n for n in os.listdir(e.cfg.download_dir))
        await e.down()
    run(main())


def test_stale_job_dir_sweep(tmp_path):
    """Job dirs a worker made (run marker) untouched for the age limit go; a
    fresh one, one a worker holds (flock), spare pools and live workers'
    recent trash stay; a dead worker's half-deleted trash goes, and so does
    trash past the grace whatever its pid (another container's pid
    namespace).  A dir without a marker (an operator's data, a reference
    deployment's finished download) is never taken."""
    import fcntl
    import subprocess
    from tritondl.service import sweep_stale_job_dirs
    base = tmp_path / "downloading"
    old, fresh, held, foreign = base / "old", base / "fresh", base / "held", base / "foreign"
    for d in (old / "sub", fresh, held, foreign, base / ".tritondl-spare-1"):
        os.makedirs(d)
    (old / "sub" / "part.mkv").write_bytes(b"x")
    (old / ".tritondl-job").write_bytes(b"")          # a failed job's dir, waiting for a retry
    (held / "f.mkv").write_bytes(b"y")
    (held / ".tritondl-running").write_bytes(b"")     # a run in progress
    (fresh / ".tritondl-job").write_bytes(b"")
    (foreign / "movie.mkv").write_bytes(b"z")
    t_old = time.time() - 10 * 86400
    for p in (old / "sub" / "part.mkv", old / "sub", old / ".tritondl-job", old, held / "f.mkv",
              held / ".tritondl-running", held, foreign / "movie.mkv", foreign):
        os.utime(p, (t_old, t_old))
    dead = subprocess.Popen(["true"])
    dead.wait()
    os.makedirs(base / f"gone.deleting-{dead.pid}-abc")
    os.makedirs(base / f"busy.deleting-{os.getpid()}-abc")
    stuck = base / f"stuck.deleting-{os.getpid()}-abc"   # "alive" pid, but untouched for 2 h
    os.makedirs(stuck)
    os.utime(stuck, (time.time() - 7200, time.time() - 7200))
    # a media id that merely looks like trash, with its job running: never taken
    odd = base / f"id.deleting-{dead.pid}-x"
    os.makedirs(odd)
    fd = os.open(held, os.O_RDONLY | os.O_DIRECTORY)
    fcntl.flock(fd, fcntl.LOCK_EX)
    fd2 = os.open(odd, os.O_RDONLY | os.O_DIRECTORY)
    fcntl.flock(fd2, fcntl.LOCK_EX)
    try:
        out = sweep_stale_job_dirs(str(base), 7 * 86400)
    finally:
        os.close(fd)
        os.close(fd2)
    assert odd.exists()
    shutil.rmtree(odd)
    names = sorted(os.path.basename(p) for p in out)
    assert names == [f"gone.deleting-{dead.pid}-abc", f"old.deleting-{os.getpid()}-stale",
                     f"stuck.deleting-{os.getpid()}-abc"]
    assert not old.exists() and fresh.exists() and held.exists() and (base / ".tritondl-spare-1").exists()
    assert (foreign / "movie.mkv").exists()
    assert (base / f"busy.deleting-{os.getpid()}-abc").exists()
    for p in out:                                    # the reaper's part
        shutil.rmtree(p)
    # the lock released, the held dir is taken on the next sweep
    assert [os.path.basename(p) for p in sweep_stale_job_dirs(str(base), 7 * 86400)] == \
        [f"held.deleting-{os.getpid()}-stale"]


def test_service_sweeps_stale_job_dirs_at_start(tmp_path):
    async def main():
        base = tmp_path / "downloading"
        os.makedirs(base / "ancient")
        os.makedirs(base / "operator-data")
        (base / "ancient" / ".tritondl-running").write_bytes(b"")    # a worker died in it long ago
        t_old = time.time() - 30 * 86400
        for p in (base / "ancient" / ".tritondl-running", base / "ancient", base / "operator-data"):
            os.utime(p, (t_old, t_old))
        e = await Env().up(tmp_path, cleanup=True, stale_job_days=7.0)
        for _ in range(100):
            if not any(n.startswith("ancient") for n in os.listdir(base)):
                break
            await asyncio.sleep(0.02)
        assert not any(n.startswith("ancient") for n in os.listdir(base))
        assert (base / "operator-data").is_dir()
        await e.down()
    run(main())


def test_long_job_hands_its_buffered_delivery_to_an_idle_worker(tmp_path):
    """Head-of-line blocking: worker A runs a slow download and holds the
    other shard's delivery in its buffer (prefetch 1 per shard, as the
    reference).  After TRITONDL_HANDBACK seconds A gives it back; idle worker
    B runs it and finishes while A's long job is still downloading.  A
    consumes again once its slot frees."""
    async def main():
        e = await Env().up(tmp_path / "a", handback_s=0.4, concurrency=1)   # every slot busy
        e.origin.rate = 1_500_000                         # the 4.5 MB job takes ~3 s
        long_url = e.origin.add("/long.mkv", os.urandom(4_500_000))
        short_url = e.origin.add("/short.mkv", os.urandom(30_000))
        e.submit(Media(id="long", source_uri=long_url), i=0)
        e.submit(Media(id="short", source_uri=short_url), i=1)
        for _ in range(100):                              # A took one and buffers the other
            if not e.svc.amqp._out.empty():
                break
            await asyncio.sleep(0.02)
        assert not e.svc.amqp._out.empty()
        cfg_b = Config()
        for k in ("retry_delay_s", "progress_log_interval_s", "heartbeat_s"):
            setattr(cfg_b, k, getattr(e.cfg, k))
        cfg_b.download_dir = str(tmp_path / "b" / "downloading")
        b = Service(cfg_b, amqp=Client(e.broker.url, heartbeat=0, retry_delay=0),
                    dispatcher=Dispatcher(cfg_b.download_dir, [HTTPDownloader(progress_interval=0.05)], 0),
                    uploader=Uploader(cfg_b.bucket, S3Client(e.s3.endpoint, Static("ak", "sk"))))
        await b.start()
        t0 = time.monotonic()
        while not b.results:
            assert time.monotonic() - t0 < 10, "the buffered job never reached the idle worker"
            await asyncio.sleep(0.02)
        assert b.results[0].ok and not e.svc.results            # B finished while A still downloads
        assert e.svc.metrics.get("jobs_handed_back") == 1 and e.svc.amqp.paused
        assert e.svc.amqp.health(0.0)[0]                         # paused on purpose is not an outage
        assert "tritondl_consumers_paused 1.0" in e.svc.metrics.render()
        res = await e.wait_results(1, timeout=20)
        assert res[0].ok
        for _ in range(250):                              # resume() re-consumes shard by shard
            if not e.svc.amqp.paused and all(sh.active for sh in e.svc.amqp.shards.values()):
                break
            await asyncio.sleep(0.02)
        assert not e.svc.amqp.paused and all(sh.active for sh in e.svc.amqp.shards.values())
        assert {c.media.id for c in e.converts()} == {"long", "short"} and e.broker.unacked_count() == 0
        await b.shutdown(grace=5)
        await e.down()
    run(main())
