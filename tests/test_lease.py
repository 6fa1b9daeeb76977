"""Job leases: a long job runs exactly once across workers, whatever the
broker's ``consumer_timeout``.

RabbitMQ (3.8.15+) closes the channel of a delivery left unacked longer than
``consumer_timeout`` (30 min by default) and requeues it.  The reference held
every delivery unacked for its whole job (``cmd/downloader/downloader.go:
103-155``, ``internal/rabbitmq/client.go:360-373``), so any torrent longer
than that ran again on another worker.  Here a job still running after
``lease_after_s`` is *leased*: the broker keeps a copy in a per-job queue
``<shard>.lease.<token>.<n>`` (``x-message-ttl`` = lease, dead-lettered back
to the shard) and the original is acked.  The copy is renewed every lease/2
and deleted when the job settles; a worker that dies stops renewing, and the
copy returns once its TTL runs out."""

import asyncio
import json
import os
import signal
import subprocess
import sys
import time

from tritondl.amqp.client import LEASE_RETURNS, Client
from tritondl.amqp.codec import Properties
from tritondl.models import Download, Media
from tritondl.s3.uploader import object_key
from tritondl.utils.backoff import ExponentialBackoff
from tritondl_testkit.fakes.broker import Broker
from tritondl_testkit.fakes.origin import Origin
from tritondl_testkit.fakes.s3 import FakeS3

from .test_permissions import Env, run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lease_queues(b: Broker) -> list[str]:
    return sorted(q for q in b.queues if ".lease." in q)


async def _client(b: Broker, url: str | None = None) -> Client:
    cl = Client(url or b.url, prefetch=1, heartbeat=0, backoff=ExponentialBackoff(initial=0.02, max_interval=0.1))
    await cl.connect()
    await cl.consume("t")
    return cl


def test_lease_acks_the_original_renews_and_releases():
    async def main():
        b = await Broker().start()
        b.consumer_timeout = 0.3
        cl = await _client(b)
        b.inject("t", "t-0", b"job", Properties(delivery_mode=2, headers={"X-Retries": 1}))
        d = await cl.get(timeout=5)
        d.hold(0.05, 0.4)
        await asyncio.sleep(0.15)
        assert d.lease is not None and b.unacked_count() == 0      # the original is acked
        q0 = d.lease.queue
        assert _lease_queues(b) == [q0] and b.queue_depth(q0) == 1
        assert q0.startswith("t-0.lease.")
        copy = b.queues[q0].messages[0]
        assert copy.body == b"job" and copy.props.headers["X-Retries"] == 1
        assert b.queues[q0].arguments["x-message-ttl"] == 400
        assert b.queues[q0].arguments["x-dead-letter-routing-key"] == "t-0"
        await asyncio.sleep(1.0)                                  # past the TTL and the consumer timeout
        assert cl.lease_stats["renewed"] >= 2 and d.lease.queue != q0
        assert len(_lease_queues(b)) == 1 and b.queue_depth("t-0") == 0
        assert b.stats["consumer_timeouts"] == 0
        assert await d.ack() is True
        assert _lease_queues(b) == [] and cl.lease_stats["released"] == 1
        await asyncio.sleep(0.6)
        assert b.queue_depth("t-0") == 0 and b.stats["expired"] == 0   # nothing came back
        await cl.close()
        await b.stop()
    run(main())


def test_a_settled_delivery_is_never_leased_and_a_short_job_costs_nothing():
    async def main():
        b = await Broker().start()
        cl = await _client(b)
        b.inject("t", "t-0", b"job")
        d = await cl.get(timeout=5)
        d.hold(0.2, 1.0)
        await d.ack()
        await asyncio.sleep(0.4)
        assert _lease_queues(b) == [] and d.lease is None and d._hold is None
        assert cl.lease_stats["taken"] == 0
        await cl.close()
        await b.stop()
    run(main())


def test_a_dead_holder_s_lease_runs_out_and_the_job_comes_back():
    """The holder stops renewing (its connection dies): the copy expires and
    dead-letters to the shard queue, marked as a lease return."""
    async def main():
        b = await Broker().start()
        cl = await _client(b)
        b.inject("t", "t-1", b"job", Properties(delivery_mode=2))
        d = await cl.get(timeout=5)
        d.hold(0.01, 0.3)
        await asyncio.sleep(0.1)
        assert d.lease is not None
        d._hold.cancel()                               # the worker "dies": no renewals, no release
        cl._closing = True
        cl.conn._abort(ConnectionError("killed"))
        await asyncio.sleep(0.5)
        assert b.queue_depth("t-1") == 1
        back = b.queues["t-1"].messages[0]
        assert back.body == b"job" and not back.redelivered
        cl2 = await _client(b)
        d2 = await cl2.get(timeout=5)
        assert d2.lease_return and d2.lease_returns == 1 and d2.maybe_duplicate
        assert d2.retry_props(0).headers[LEASE_RETURNS] == 1
        await d2.ack()
        await cl2.close()
        await b.stop()
    run(main())


def test_shutdown_gives_a_leased_job_back_at_once():
    async def main():
        b = await Broker().start()
        cl = await _client(b)
        b.inject("t", "t-0", b"job", Properties(delivery_mode=2, headers={"X-Retries": 2}))
        d = await cl.get(timeout=5)
        d.hold(0.01, 30.0)
        await asyncio.sleep(0.1)
        assert d.lease is not None
        await cl.close()
        assert _lease_queues(b) == [] and b.queue_depth("t-0") == 1     # back now, not in 30 s
        m = b.queues["t-0"].messages[0]
        assert m.props.headers["X-Retries"] == 2 and LEASE_RETURNS not in m.props.headers
        assert cl.lease_stats["requeued"] == 1
        await b.stop()
    run(main())


def test_a_lease_the_broker_refuses_falls_back_to_holding_the_delivery():
    """A user without configure on the lease queues: the delivery is held
    unacked, as the reference did; the refusal is remembered per shard."""
    async def main():
        b = await Broker().start()
        b.add_user("ref", "pw", configure=r"^t(-\d+)?$", write=r"^t(-\d+)?$", read=r"^t(-\d+)?$")
        cl = await _client(b, f"amqp://ref:pw@{b.host}:{b.port}/")
        b.inject("t", "t-0", b"job")
        d = await cl.get(timeout=5)
        d.hold(0.01, 1.0)
        await asyncio.sleep(0.2)
        assert d.lease is None and "t-0" in cl._lease_refused and cl.lease_stats["refused"] == 1
        assert b.unacked_count() == 1
        assert await d.ack() is True
        await asyncio.sleep(0.05)
        assert b.unacked_count() == 0
        b.inject("t", "t-0", b"job2")
        d2 = await cl.get(timeout=5)
        d2.hold(0.01, 1.0)
        assert d2._hold_timer is None                    # not even tried again
        await d2.ack()
        await cl.close()
        await b.stop()
    run(main())


def test_busy_hand_back_delay_doubles_up_to_the_cap(tmp_path):
    async def main():
        e = await Env().up(tmp_path, retry_delay_s=0.5, retry_delay_max_s=4.0)
        assert [e.svc.busy_delay(n) for n in range(5)] == [1.0, 2.0, 4.0, 4.0, 4.0]
        await e.down()
    run(main())


def _worker_env(b, s3, download_dir, **extra):
    env = dict(os.environ, RABBITMQ_ENDPOINT=b.endpoint, RABBITMQ_USERNAME="guest", RABBITMQ_PASSWORD="guest",
               S3_ENDPOINT=s3.endpoint, PYTHONPATH=ROOT, TRITONDL_BT_DHT="0", LOG_LEVEL="info", LOG_FORMAT="json",
               TRITONDL_PROGRESS_LOG_INTERVAL="0", TRITONDL_GPU_VERIFY="off", TRITONDL_RETRY_DELAY="0.5",
               TRITONDL_DOWNLOAD_DIR=str(download_dir))
    env.update({k: str(v) for k, v in extra.items()})
    return env


def _log_lines(path) -> list[dict]:
    out = []
    with open(path) as f:
        for line in f:
            try:
                out.append(json.loads(line))
            except ValueError:
                pass
    return out


async def _two_workers(tmp_path, shared: bool, consumer_timeout: float = 0.3):
    b = await Broker().start()
    b.consumer_timeout = consumer_timeout
    o = await Origin().start()
    s3 = await FakeS3().start()
    data = os.urandom(3_000_000)
    o.rate = 1_000_000                                # a 3 s job: ten consumer timeouts long
    url = o.add("/long.mkv", data)
    b.declare("v1.download")
    procs, logs = [], []
    for i in range(2):
        dd = tmp_path / ("downloading" if shared else f"node{i}") / ("" if shared else "downloading")
        log_path = tmp_path / f"worker{i}.log"
        logs.append(log_path)
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "tritondl"], cwd=str(tmp_path),
            env=_worker_env(b, s3, dd, TRITONDL_LEASE_AFTER="0.1", TRITONDL_LEASE="1.0"),
            stdout=subprocess.DEVNULL, stderr=open(log_path, "w")))
    return b, o, s3, data, url, procs, logs


def _gets(o, path="/long.mkv"):
    return [r for r in o.requests if r[0] == "GET" and r[1] == path]


def _converts(b):
    return [m for q in ("v1.convert-0", "v1.convert-1") for m in (b.queues[q].messages if q in b.queues else [])]


async def _wait_consumers(b, n, timeout=60):
    t0 = time.monotonic()
    while sum(len(b.queues[q].consumers) for q in ("v1.download-0", "v1.download-1") if q in b.queues) < n:
        assert time.monotonic() - t0 < timeout, "workers did not start consuming"
        await asyncio.sleep(0.05)


def _check_two_worker_run(tmp_path, shared: bool):
    async def main():
        b, o, s3, data, url, procs, logs = await _two_workers(tmp_path, shared)
        try:
            await _wait_consumers(b, 4)
            b.inject("v1.download", "v1.download-0",
                     Download(created_at="t", media=Media(id="long", source_uri=url)).encode(),
                     Properties(delivery_mode=2))
            t0 = time.monotonic()
            while not _converts(b):
                assert time.monotonic() - t0 < 60 and all(p.poll() is None for p in procs)
                await asyncio.sleep(0.05)
            await asyncio.sleep(1.5)                     # past a lease TTL: nothing comes back
            assert len(_gets(o)) == 1, _gets(o)          # one origin download
            assert len(_converts(b)) == 1                # one v1.convert
            assert s3.object_bytes("triton-staging", object_key("long", "long.mkv")) == data
            assert b.stats["consumer_timeouts"] == 0
            assert _lease_queues(b) == [] and b.unacked_count() == 0
            assert b.queue_depth("v1.download-0") == 0 and b.queue_depth("v1.download-1") == 0
        finally:
            for p in procs:
                p.send_signal(signal.SIGTERM)
            for p in procs:
                p.wait(timeout=30)
        lines = [ln for path in logs for ln in _log_lines(path)]
        assert any("job leased" in ln.get("msg", "") for ln in lines)
        # no worker spent a job slot waiting on a lock
        assert not [ln for ln in lines if "waiting for it" in ln.get("msg", "") or
                    "handing the delivery back" in ln.get("msg", "")]
        await s3.stop()
        await o.stop()
        await b.stop()
    asyncio.run(asyncio.wait_for(main(), 150))


def test_two_workers_sharing_a_download_dir_run_a_long_job_once(tmp_path):
    _check_two_worker_run(tmp_path, shared=True)


def test_two_nodes_run_a_long_job_once(tmp_path):
    _check_two_worker_run(tmp_path, shared=False)


def test_a_leased_job_whose_worker_dies_runs_again_elsewhere_and_is_counted(tmp_path):
    """Worker A leases the job and is SIGKILLed: its copy expires after the
    lease and worker B (another node) runs the job, which arrives with
    X-Lease-Returns 1."""
    async def main():
        b = await Broker().start()
        o = await Origin().start()
        s3 = await FakeS3().start()
        data = os.urandom(2_000_000)
        o.rate = 2_000_000
        url = o.add("/k.mkv", data)
        b.declare("v1.download")
        env_a = _worker_env(b, s3, tmp_path / "a", TRITONDL_LEASE_AFTER="0.1", TRITONDL_LEASE="1.0")
        a = subprocess.Popen([sys.executable, "-m", "tritondl"], cwd=str(tmp_path), env=env_a,
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        try:
            await _wait_consumers(b, 2)
            b.inject("v1.download", "v1.download-1",
                     Download(created_at="t", media=Media(id="k", source_uri=url)).encode(),
                     Properties(delivery_mode=2))
            t0 = time.monotonic()
            while not (_lease_queues(b) and b.queue_depth(_lease_queues(b)[0]) and not b.unacked_count()):
                assert time.monotonic() - t0 < 30           # the copy is in place and the original acked
                await asyncio.sleep(0.02)
            os.kill(a.pid, signal.SIGKILL)
            a.wait()
            t_kill = time.monotonic()
            assert b.unacked_count() == 0 and b.queue_depth("v1.download-1") == 0
            while not b.queue_depth("v1.download-1"):
                assert time.monotonic() - t_kill < 5
                await asyncio.sleep(0.02)
            back = b.queues["v1.download-1"].messages[0]
            assert back.props.headers["x-death"][0]["reason"] == "expired"
            env_b = _worker_env(b, s3, tmp_path / "b", TRITONDL_LEASE_AFTER="0.1", TRITONDL_LEASE="1.0")
            bw = subprocess.Popen([sys.executable, "-m", "tritondl"], cwd=str(tmp_path), env=env_b,
                                  stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            try:
                while not _converts(b):
                    assert time.monotonic() - t_kill < 60 and bw.poll() is None
                    await asyncio.sleep(0.05)
                assert s3.object_bytes("triton-staging", object_key("k", "k.mkv")) == data
                assert len(_converts(b)) == 1 and len(_gets(o, "/k.mkv")) == 2
                await asyncio.sleep(0.2)
                # A's expired lease queue lingers empty until its x-expires; B's is gone
                assert all(b.queue_depth(q) == 0 for q in _lease_queues(b)) and b.unacked_count() == 0
                assert len(_lease_queues(b)) <= 1
            finally:
                bw.terminate()
                bw.wait(timeout=30)
        finally:
            if a.poll() is None:
                a.kill()
        await s3.stop()
        await o.stop()
        await b.stop()
    asyncio.run(asyncio.wait_for(main(), 150))


def test_a_duplicate_of_a_running_job_is_handed_back_at_once_and_acked_after(tmp_path):
    """A copy of a running job comes back (redelivered: an earlier holder's
    channel died) while a worker on a shared download dir runs it.  The
    worker that gets the copy finds the job held (flock, or the in-process
    lock if it is the same worker: two job slots each, so the copy is never
    just buffered behind the run), hands the copy back within a second
    (X-Busy, growing delay) instead of waiting out the run, and acks it
    without running it once the job has finished (the node's done-ledger)."""
    async def main():
        b = await Broker().start()
        o = await Origin().start()
        s3 = await FakeS3().start()
        data = os.urandom(2_000_000)
        o.rate = 1_000_000
        url = o.add("/dup.mkv", data)
        b.declare("v1.download")
        dd = tmp_path / "downloading"
        procs, logs = [], []
        for i in range(2):
            logs.append(tmp_path / f"w{i}.log")
            procs.append(subprocess.Popen(
                [sys.executable, "-m", "tritondl"], cwd=str(tmp_path),
                env=_worker_env(b, s3, dd, TRITONDL_RETRY_DELAY="1", TRITONDL_LEASE_AFTER="0.2",
                                TRITONDL_LEASE="2", TRITONDL_CONCURRENCY="2"),
                stdout=subprocess.DEVNULL, stderr=open(logs[-1], "w")))
        try:
            await _wait_consumers(b, 4)
            body = Download(created_at="t", media=Media(id="dup", source_uri=url)).encode()
            b.inject("v1.download", "v1.download-0", body, Properties(delivery_mode=2))
            t0 = time.monotonic()
            while not _gets(o, "/dup.mkv"):
                assert time.monotonic() - t0 < 30
                await asyncio.sleep(0.02)
            b.pause_delivery(True)
            b.inject("v1.download", "v1.download-1", body, Properties(delivery_mode=2))
            b.queues["v1.download-1"].messages[-1].redelivered = True
            b.pause_delivery(False)
            while len(_converts(b)) < 1:
                assert time.monotonic() - t0 < 60 and all(p.poll() is None for p in procs)
                await asyncio.sleep(0.05)
            # the handed-back copy comes round again and is recognised
            t1 = time.monotonic()
            while True:
                lines = [ln for path in logs for ln in _log_lines(path)]
                if any("already completed on this node" in ln.get("msg", "") for ln in lines):
                    break
                assert time.monotonic() - t1 < 30
                await asyncio.sleep(0.1)
            await asyncio.sleep(0.3)
            assert len(_gets(o, "/dup.mkv")) == 1 and len(_converts(b)) == 1
            assert b.unacked_count() == 0 and _lease_queues(b) == []
            assert all(b.queue_depth(q) == 0 for q in b.queues if q.startswith("v1.download-"))
        finally:
            for p in procs:
                p.send_signal(signal.SIGTERM)
            for p in procs:
                p.wait(timeout=30)
        lines = [ln for path in logs for ln in _log_lines(path)]
        back = [ln for ln in lines if "handing the delivery back" in ln.get("msg", "")]
        assert back and back[0]["busy"] == 1 and float(back[0]["delay_s"]) == 1.0
        waits = [ln for ln in lines if "waiting for it" in ln.get("msg", "")]
        for w in waits:                                   # every lock wait ended within a second
            t_w = w["time"]
            assert any(bk["time"] >= t_w for bk in back)
        await s3.stop()
        await o.stop()
        await b.stop()
    asyncio.run(asyncio.wait_for(main(), 150))


def test_a_duplicate_in_another_slot_of_the_same_worker_is_handed_back(tmp_path):
    async def main():
        e = await Env().up(tmp_path, concurrency=2, retry_delay_s=0.2, retry_delay_max_s=1.0)
        data = os.urandom(1_500_000)
        e.origin.rate = 1_000_000
        url = e.origin.add("/same.mkv", data)
        e.submit(Media(id="same", source_uri=url), 0)
        e.submit(Media(id="same", source_uri=url), 1)
        t0 = time.monotonic()
        res = await e.wait_results(3, timeout=30)
        busy = [r for r in res if r.stage == "lock"]
        assert busy and all(r.seconds < 1.0 for r in busy), res
        assert [r.stage for r in res if r.stage != "lock"] == ["done", "duplicate"], res
        assert len(_gets(e.origin, "/same.mkv")) == 1 and len(e.converts()) == 1
        assert time.monotonic() - t0 < 10
        await e.down()
    run(main())


async def _restart(e):
    """A new worker process on the same broker, origin, S3 and download dir."""
    from tritondl.fetch.http import HTTPDownloader
    from tritondl.fetch.registry import Dispatcher
    from tritondl.s3.client import S3Client
    from tritondl.s3.credentials import Static
    from tritondl.s3.uploader import Uploader
    from tritondl.service import Service
    e.amqp = Client(e.broker.url, heartbeat=0, retry_delay=0, backoff=ExponentialBackoff(initial=0.02, max_interval=0.1))
    e.svc = Service(e.cfg, amqp=e.amqp,
                    dispatcher=Dispatcher(e.cfg.download_dir, [HTTPDownloader(progress_interval=0.05, max_retries=1)], 0),
                    uploader=Uploader(e.cfg.bucket, S3Client(e.s3.endpoint, Static("ak", "sk"))))
    await e.svc.start()


def test_graceful_restarts_and_connection_drops_do_not_count_as_crashes(tmp_path):
    """the redelivery limit counts only returns of runs that never
    settled (the run marker is still in the job dir).  A job interrupted by
    a graceful shutdown, and a buffered delivery returned by a connection
    drop, come back redelivered but are not counted; a crashed run is."""
    from tritondl.utils import ledger as jobdir

    async def main():
        e = await Env().up(tmp_path, redelivery_limit=1, lease_after_s=0)
        e.origin.rate = 1_000_000
        data = os.urandom(3_000_000)
        url = e.origin.add("/g.mkv", data)
        e.submit(Media(id="g", source_uri=url), 0)
        t0 = time.monotonic()
        while not _gets(e.origin, "/g.mkv"):
            assert time.monotonic() - t0 < 10
            await asyncio.sleep(0.02)
        jd = os.path.join(e.cfg.download_dir, "g")
        assert jobdir.was_running(jd)
        await e.svc.shutdown(grace=0.1)                # SIGTERM: the run is cancelled, not crashed
        assert not jobdir.was_running(jd) and jobdir.is_ours(jd)
        for _ in range(2):                             # buffered deliveries, connection dropped
            cl = await Client(e.broker.url, heartbeat=0, retry_delay=0).connect()
            await cl.consume("v1.download")
            d = await cl.get(timeout=5)
            assert d.redelivered
            cl._closing = True
            cl.conn._abort(ConnectionError("dropped"))
            await asyncio.sleep(0.05)
        e.origin.rate = None
        await _restart(e)
        res = await e.wait_results(1, timeout=20)
        assert res[0].stage == "done", res            # three returns, none of them a crash
        assert len(e.converts()) == 1
        assert not os.path.exists(os.path.join(jd, ".tritondl-redeliveries"))
        await e.down()
    run(main())


def test_a_resubmitted_job_interrupted_mid_run_runs_again(tmp_path):
    """The same body was submitted again after this node finished it once
    (its done-ledger entry is still inside the TTL).  The second run is
    interrupted; its redelivered copy must run, not be acked as already
    done: the entry is dropped when a fresh submission starts."""
    async def main():
        e = await Env().up(tmp_path, lease_after_s=0)
        data = os.urandom(3_000_000)
        url = e.origin.add("/again.mkv", data)
        body = Download(created_at="t", media=Media(id="again", source_uri=url)).encode()
        e.svc.ledger.add(body)                           # the first submission finished earlier
        e.origin.rate = 1_000_000
        e.broker.inject("v1.download", "v1.download-0", body, Properties(delivery_mode=2))
        t0 = time.monotonic()
        while not _gets(e.origin, "/again.mkv"):
            assert time.monotonic() - t0 < 10
            await asyncio.sleep(0.02)
        assert not e.svc.ledger.has(body)
        await e.svc.shutdown(grace=0.1)                  # the run is cut short; the delivery goes back
        e.origin.rate = None
        await _restart(e)
        res = await e.wait_results(1, timeout=20)
        assert res[0].stage == "done", res
        assert len(_gets(e.origin, "/again.mkv")) >= 2 and len(e.converts()) == 1
        assert e.svc.ledger.has(body)
        assert e.s3.object_bytes("triton-staging", object_key("again", "again.mkv")) == data
        await e.down()
    run(main())


def test_a_crashed_run_is_counted(tmp_path):
    async def main():
        e = await Env().up(tmp_path, redelivery_limit=1, lease_after_s=0)
        url = e.origin.add("/c.mkv", os.urandom(10_000))
        body = Download(created_at="t", media=Media(id="c", source_uri=url)).encode()
        jd = os.path.join(e.cfg.download_dir, "c")
        os.makedirs(jd)
        with open(os.path.join(jd, ".tritondl-redeliveries"), "w") as f:
            f.write("1")
        open(os.path.join(jd, ".tritondl-running"), "w").close()    # the last run died mid-job
        e.broker.pause_delivery(True)
        e.broker.inject("v1.download", "v1.download-0", body, Properties(delivery_mode=2))
        e.broker.queues["v1.download-0"].messages[-1].redelivered = True
        e.broker.pause_delivery(False)
        res = await e.wait_results(1)
        assert res[0].stage == "redelivery-limit", res
        assert not _gets(e.origin, "/c.mkv")
        await e.down()
    run(main())


def test_lease_returns_from_other_nodes_count_towards_the_limit(tmp_path):
    async def main():
        e = await Env().up(tmp_path, redelivery_limit=2)
        url = e.origin.add("/n.mkv", os.urandom(10_000))
        body = Download(created_at="t", media=Media(id="n", source_uri=url)).encode()
        death = [{"queue": "v1.download-0.lease.abc.3", "reason": "expired", "count": 1,
                  "exchange": "", "routing-keys": ["v1.download-0.lease.abc.3"]}]
        e.broker.inject("v1.download", "v1.download-0", body,
                        Properties(delivery_mode=2, headers={LEASE_RETURNS: 2, "x-death": death}))
        res = await e.wait_results(1)
        assert res[0].stage == "redelivery-limit", res       # third return > 2
        dead = [m for q in ("v1.download.dead-0", "v1.download.dead-1") for m in
                (e.broker.queues[q].messages if q in e.broker.queues else [])]
        assert len(dead) == 1 and not _gets(e.origin, "/n.mkv")
        await e.down()
    run(main())


def test_a_leased_job_survives_a_broker_connection_drop(tmp_path):
    """The connection drops while a leased job runs: the lease copy sits in
    its durable queue, the worker reconnects, keeps renewing, finishes the
    job and deletes the copy.  Nothing comes back and nothing is redelivered."""
    async def main():
        e = await Env().up(tmp_path, lease_after_s=0.1, lease_s=1.0)
        e.origin.rate = 1_000_000
        data = os.urandom(2_500_000)
        url = e.origin.add("/drop.mkv", data)
        e.submit(Media(id="drop", source_uri=url))
        t0 = time.monotonic()
        while not e.amqp.lease_stats["taken"]:
            assert time.monotonic() - t0 < 10
            await asyncio.sleep(0.02)
        await e.broker.drop_connections()
        res = await e.wait_results(1, timeout=30)
        assert res[0].ok, res
        await asyncio.sleep(1.5)                          # past a TTL: nothing returns
        assert all(e.broker.queue_depth(q) == 0 for q in e.broker.queues if q.startswith("v1.download"))
        assert e.amqp.lease_stats["released"] == 1 and e.amqp.lease_stats["lost"] == 0
        assert len(_gets(e.origin, "/drop.mkv")) == 1 and len(e.converts()) == 1
        await e.down()
    run(main())


def test_a_job_parked_past_the_consumer_timeout_is_leased(tmp_path):
    """A failed job parked in-process (the broker refused its delay queue)
    waits retry_delay_max_s unacked: the lease keeps consumer_timeout away
    from it too, and the parked retry still goes out after the wait."""
    from .test_permissions import REF_PERMS

    async def main():
        # the reference's permissions plus what a lease needs: configure and read on the lease
        # queues (a queue with a dead-letter exchange needs read), write on the default exchange
        perms = dict(REF_PERMS, configure=r"^v1\.download(-\d+)?(\.lease\..*)?$",
                     read=r"^v1\.download(-\d+)?(\.lease\..*)?$",
                     write=r"^(v1\.download(-\d+)?|v1\.convert|amq\.default)$")
        e = await Env().up(tmp_path, user="ref", perms=perms, lease_after_s=0.1, lease_s=1.0, retry_delay_s=1.5,
                           max_retries=1)
        e.amqp.lease_after, e.amqp.lease_ttl = 0.1, 1.0
        e.broker.consumer_timeout = 0.5
        e.submit(Media(id="pk", source_uri=e.origin.url("/missing.mkv")))
        res = await e.wait_results(2, timeout=30)
        assert [r.ok for r in res] == [False, False]
        assert e.amqp.parked_total >= 1 and e.amqp.lease_stats["taken"] >= 1
        assert e.broker.stats["consumer_timeouts"] == 0
        await e.down()
    run(main())
