"""Chaos soak: jobs flow while faults fire at random — broker connection
drops, publish nacks, flow-control blocks, S3 5xx bursts and origin
connection cuts.  Invariant (at-least-once): every job
ends with its object in S3 and at least one ``v1.convert`` for it, and no
delivery is left unacked."""

import asyncio
import random

import pytest

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
from tritondl.utils.backoff import ExponentialBackoff
from tritondl.utils.config import Config


@pytest.mark.parametrize("seed", [1234, 7, 99, 2024, 31337])
def test_chaos_soak_every_job_lands(tmp_path, seed):
    rng = random.Random(seed)
    n_jobs = 60

    async def main():
        broker = await Broker().start()
        origin = await Origin().start()
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        cfg = Config()
        cfg.download_dir = str(tmp_path / "dl")
        cfg.retry_delay_s = 0
        cfg.max_retries = 50            # faults are transient: keep retrying
        cfg.concurrency = 3
        cfg.prefetch = 3
        cfg.progress_log_interval_s = 0
        cfg.heartbeat_s = 0
        cfg.cleanup = True
        http = HTTPDownloader(progress_interval=0.05, max_retries=3)
        svc = Service(cfg, amqp=Client(broker.url, prefetch=3, heartbeat=0, retry_delay=0,
                                       backoff=ExponentialBackoff(initial=0.01, max_interval=0.05)),
                      dispatcher=Dispatcher(cfg.download_dir, [http], 0),
                      uploader=Uploader(cfg.bucket, S3Client(s3.endpoint, Static("ak", "sk"), max_retries=2,
                                                             part_size=5 << 20, multipart_threshold=6 << 20)))
        await svc.start()
        origin.rate = 40_000_000          # ~2-3 s of traffic so faults land mid-job
        sizes = {}
        for i in range(n_jobs):
            size = rng.choice([1, 50_000, 700_000, 7_000_000])
            data = bytes([i % 251]) * size
            sizes[i] = size
            url = origin.add(f"/m/job{i}.mkv", data)
            body = Download(created_at="t", media=Media(id=f"c{i}", source_uri=url)).encode()
            broker.inject("v1.download", f"v1.download-{i % 2}", body, Properties(delivery_mode=2))

        stop = asyncio.Event()
        fired = {"drop": 0, "nack": 0, "block": 0, "s3": 0, "cut": 0, "unbind": 0, "complete200": 0}

        async def chaos():
            while not stop.is_set():
                await asyncio.sleep(rng.uniform(0.05, 0.25))
                f = rng.choice(list(fired))
                fired[f] += 1
                if f == "drop":
                    await broker.drop_connections()
                elif f == "nack":
                    broker.fail_next_publishes(1)
                elif f == "block":
                    broker.set_blocked(True)
                    await asyncio.sleep(0.05)
                    broker.set_blocked(False)
                elif f == "s3":
                    s3.fail_next(2, 503)
                elif f == "unbind":
                    # v1.convert's binding removed: publishes come back (mandatory) and the
                    # worker binds the queue again instead of losing the Convert
                    broker.unbind_queue(f"v1.convert-{rng.randrange(2)}")
                elif f == "complete200":
                    s3.complete_error_200 = 1        # S3's 200-with-<Error> CompleteMultipartUpload
                else:
                    origin.cut_after, origin.cut_times = 200_000, 1
        chaos_task = asyncio.ensure_future(chaos())

        def landed():
            objs = s3.buckets.get("triton-staging", {})
            return [i for i in range(n_jobs) if object_key(f"c{i}", f"job{i}.mkv") in objs]

        for _ in range(1500):
            if len(landed()) == n_jobs:
                break
            await asyncio.sleep(0.05)
        stop.set()
        await chaos_task
        broker.set_blocked(False)
        # every job's Convert is eventually published (duplicates allowed)
        for _ in range(400):
            conv = {Convert.decode(m.body).media.id
                    for q in ("v1.convert-0", "v1.convert-1") if q in broker.queues
                    for m in list(broker.queues[q].messages)}
            if len(conv) == n_jobs and broker.queue_depth("v1.download-0") + broker.queue_depth("v1.download-1") == 0 \
                    and broker.unacked_count() == 0:
                break
            await asyncio.sleep(0.05)
        got = landed()
        objs = s3.buckets.get("triton-staging", {})
        settled = (broker.unacked_count(), broker.queue_depth("v1.download-0") + broker.queue_depth("v1.download-1"))
        await svc.shutdown(grace=5)
        await s3.stop()
        await origin.stop()
        await broker.stop()
        assert len(got) == n_jobs, (sorted(set(range(n_jobs)) - set(got)), fired)
        for i in range(n_jobs):
            assert objs[object_key(f"c{i}", f"job{i}.mkv")].size == sizes[i]
        assert len(conv) == n_jobs, (n_jobs - len(conv), fired)
        assert settled == (0, 0), settled          # nothing left unacked or queued
        assert sum(fired.values()) >= 8, fired
        print("chaos fired:", fired, "job results:", len(svc.results))
    asyncio.run(asyncio.wait_for(main(), 170))


def test_chaos_with_s3_outage_beyond_retry_budget_loses_nothing(tmp_path):
    """Random faults plus an S3 outage that outlasts the whole retry budget
    (delayed retries through broker TTL queues, then the dead-letter topic).
    Invariant: every job is accounted for — its object + a v1.convert, or a
    copy in the DLQ — and nothing is left unacked or waiting in a queue."""
    rng = random.Random(99)
    n_jobs = 40

    async def main():
        broker = await Broker().start()
        origin = await Origin().start()
        s3 = await FakeS3(access_key="ak", secret_key="sk").start()
        cfg = Config()
        cfg.download_dir = str(tmp_path / "dl")
        cfg.retry_delay_s = 0.05
        cfg.retry_backoff = 2.0
        cfg.max_retries = 2             # budget ≈ 0.05 + 0.1 s of delay: the outage outlasts it
        cfg.concurrency = 3
        cfg.prefetch = 3
        cfg.progress_log_interval_s = 0
        cfg.heartbeat_s = 0
        cfg.cleanup = True
        http = HTTPDownloader(progress_interval=0.05, max_retries=3)
        svc = Service(cfg, amqp=Client(broker.url, prefetch=3, heartbeat=0,
                                       backoff=ExponentialBackoff(initial=0.01, max_interval=0.05)),
                      dispatcher=Dispatcher(cfg.download_dir, [http], 0),
                      uploader=Uploader(cfg.bucket, S3Client(s3.endpoint, Static("ak", "sk"), max_retries=0,
                                                             part_size=5 << 20, multipart_threshold=6 << 20)))
        await svc.start()
        origin.rate = 40_000_000
        for i in range(n_jobs):
            size = rng.choice([1, 50_000, 700_000, 3_000_000])
            url = origin.add(f"/m/job{i}.mkv", bytes([i % 251]) * size)
            body = Download(created_at="t", media=Media(id=f"c{i}", source_uri=url)).encode()
            broker.inject("v1.download", f"v1.download-{i % 2}", body, Properties(delivery_mode=2))

        stop = asyncio.Event()
        fired = {"drop": 0, "nack": 0, "s3": 0, "cut": 0, "outage": 0}

        async def chaos():
            await asyncio.sleep(0.3)
            s3.fail_for(3.0)                 # the long one
            fired["outage"] += 1
            while not stop.is_set():
                await asyncio.sleep(rng.uniform(0.1, 0.3))
                f = rng.choice(["drop", "nack", "s3", "cut"])
                fired[f] += 1
                if f == "drop":
                    await broker.drop_connections()
                elif f == "nack":
                    broker.fail_next_publishes(1)
                elif f == "s3":
                    s3.fail_next(2, 503)
                else:
                    origin.cut_after, origin.cut_times = 200_000, 1
        chaos_task = asyncio.ensure_future(chaos())

        def accounted():
            objs = s3.buckets.get("triton-staging", {})
            conv = {Convert.decode(m.body).media.id for q in ("v1.convert-0", "v1.convert-1") if q in broker.queues
                    for m in list(broker.queues[q].messages)}
            dead = {Download.decode(m.body).media.id for q in ("v1.download.dead-0", "v1.download.dead-1")
                    if q in broker.queues for m in list(broker.queues[q].messages)}
            done = {f"c{i}" for i in range(n_jobs) if object_key(f"c{i}", f"job{i}.mkv") in objs} & conv
            return done, dead

        def quiet():
            waiting = sum(len(q.messages) for name, q in broker.queues.items()
                          if name.startswith("v1.download") and ".dead" not in name)
            return waiting == 0 and broker.unacked_count() == 0

        for _ in range(2000):
            done, dead = accounted()
            if len(done | dead) == n_jobs and quiet():
                break
            await asyncio.sleep(0.05)
        stop.set()
        await chaos_task
        for _ in range(100):                 # faults stopped: let in-flight retries settle
            done, dead = accounted()
            if len(done | dead) == n_jobs and quiet():
                break
            await asyncio.sleep(0.05)
        settled = quiet()
        await svc.shutdown(grace=5)
        await s3.stop()
        await origin.stop()
        await broker.stop()
        assert len(done | dead) == n_jobs, (sorted({f"c{i}" for i in range(n_jobs)} - done - dead), fired)
        assert dead, "the outage should have dead-lettered some jobs"
        assert settled
        print("outage chaos:", fired, "done", len(done), "dead-lettered", len(dead))
    asyncio.run(asyncio.wait_for(main(), 170))
