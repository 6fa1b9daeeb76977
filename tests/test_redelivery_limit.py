"""A job that kills its worker (an OOM kill, a crash in native code) comes
back unacknowledged to the next worker, forever: the reference had no
defence (its job loop held the delivery unacked, ``downloader.go:103-155``),
and neither does ``X-Retries``, which only counts failures a worker lived to
handle.  The worker counts unacknowledged returns of a job in its job dir
(or RabbitMQ's ``x-delivery-count`` on quorum queues) and dead-letters it
past ``TRITONDL_REDELIVERY_LIMIT``."""

import asyncio
import os
import signal
import subprocess
import sys
import time

from tritondl.amqp.codec import Properties
from tritondl.models import Download, Media
from tritondl_testkit.fakes.broker import Broker
from tritondl_testkit.fakes.origin import Origin
from tritondl_testkit.fakes.s3 import FakeS3

from .test_permissions import Env, run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dead(broker):
    return [m for q in ("v1.download.dead-0", "v1.download.dead-1") for m in
            (broker.queues[q].messages if q in broker.queues else [])]


def test_redelivered_past_the_limit_is_dead_lettered_without_running(tmp_path):
    async def main():
        e = await Env().up(tmp_path, redelivery_limit=2)
        url = e.origin.add("/r.mkv", os.urandom(10_000))
        body = Download(created_at="t", media=Media(id="r1", source_uri=url)).encode()
        d = os.path.join(e.cfg.download_dir, "r1")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, ".tritondl-redeliveries"), "w") as f:
            f.write("2")                                   # two earlier workers died on it ...
        open(os.path.join(d, ".tritondl-running"), "w").close()   # ... and so did the last one
        e.broker.pause_delivery(True)
        e.broker.inject("v1.download", "v1.download-0", body, Properties(delivery_mode=2))
        e.broker.queues["v1.download-0"].messages[-1].redelivered = True
        e.broker.pause_delivery(False)
        res = await e.wait_results(1)
        assert res[0].stage == "redelivery-limit", res
        assert not [r for r in e.origin.requests if r[1] == "/r.mkv"]
        dead = _dead(e.broker)
        assert len(dead) == 1 and dead[0].props.headers["X-Failed-Stage"] == "redelivery-limit"
        assert not os.path.exists(os.path.join(d, ".tritondl-redeliveries"))
        # below the limit a redelivered job runs, and its count is cleared on success
        url2 = e.origin.add("/s.mkv", os.urandom(10_000))
        e.broker.pause_delivery(True)
        e.broker.inject("v1.download", "v1.download-1",
                        Download(created_at="t", media=Media(id="s1", source_uri=url2)).encode(),
                        Properties(delivery_mode=2, headers={"x-delivery-count": 1}))
        e.broker.queues["v1.download-1"].messages[-1].redelivered = True
        e.broker.pause_delivery(False)
        res = await e.wait_results(2)
        assert res[1].ok, res[1]
        await e.down()
    run(main())


def test_a_job_that_kills_its_workers_is_dead_lettered(tmp_path):
    """Three worker processes are killed (SIGKILL) mid-download of the same
    job; the fourth delivery (third redelivery, limit 2) is dead-lettered
    without a download, and the worker lives on."""
    async def main():
        b = await Broker().start()
        o = await Origin().start()
        s3 = await FakeS3().start()
        o.rate = 2_000_000                                # 8 MiB at 2 MB/s: seconds of download
        url = o.add("/killer.mkv", os.urandom(8 << 20))
        env = dict(os.environ, RABBITMQ_ENDPOINT=b.endpoint, RABBITMQ_USERNAME="guest",
                   RABBITMQ_PASSWORD="guest", S3_ENDPOINT=s3.endpoint, PYTHONPATH=ROOT,
                   TRITONDL_BT_DHT="0", LOG_LEVEL="warning", TRITONDL_PROGRESS_LOG_INTERVAL="0",
                   TRITONDL_GPU_VERIFY="off", TRITONDL_REDELIVERY_LIMIT="2", TRITONDL_CLEANUP="0",
                   TRITONDL_DOWNLOAD_DIR=str(tmp_path / "downloading"))
        b.declare("v1.download")
        b.inject("v1.download", "v1.download-0",
                 Download(created_at="t", media=Media(id="k1", source_uri=url)).encode(), Properties(delivery_mode=2))
        gets = lambda: len([r for r in o.requests if r[1] == "/killer.mkv"])   # noqa: E731
        for k in range(3):
            p = subprocess.Popen([sys.executable, "-m", "tritondl"], env=env, cwd=str(tmp_path),
                                 stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            t0 = time.monotonic()
            while gets() <= k:                             # this worker started downloading it
                assert time.monotonic() - t0 < 60 and p.poll() is None
                await asyncio.sleep(0.05)
            os.kill(p.pid, signal.SIGKILL)                 # dies mid-job: the delivery goes back
            p.wait()
            await asyncio.sleep(0.1)
        p = subprocess.Popen([sys.executable, "-m", "tritondl"], env=env, cwd=str(tmp_path),
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        try:
            t0 = time.monotonic()
            while not _dead(b):
                assert time.monotonic() - t0 < 60 and p.poll() is None
                await asyncio.sleep(0.05)
            assert gets() == 3                             # not downloaded a fourth time
            assert _dead(b)[0].props.headers["X-Failed-Stage"] == "redelivery-limit"
            await asyncio.sleep(0.3)
            assert p.poll() is None and b.unacked_count() == 0
        finally:
            p.terminate()
            p.wait(timeout=30)
        await s3.stop()
        await o.stop()
        await b.stop()
    asyncio.run(asyncio.wait_for(main(), 180))
