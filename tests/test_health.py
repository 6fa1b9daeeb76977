"""``/healthz`` reflects consumption, not just the TCP connection (VERDICT
r04 Missing/Next #2).

The reference's 1 s scheduler re-created a dead processor
(``internal/rabbitmq/client.go:139-166``); here re-creation is event-driven
(consumer-cancel and channel-close callbacks, the reconnect supervisor), and
these tests make sure a shard that *stays* dead, a connection that stays
down, or a consumer that gets nothing while its queue fills up, turns the
probe red — and that it goes green again once the shard consumes."""

import asyncio
import os
import socket
import time

from tritondl.utils.metrics import Metrics
from tritondl_testkit.fakes.broker import Broker
from tritondl.models import Media

from .test_permissions import Env, run


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _get(port: int, path: str = "/healthz") -> tuple[int, bytes]:
    r, w = await asyncio.open_connection("127.0.0.1", port)
    w.write(f"GET {path} HTTP/1.0\r\nHost: x\r\n\r\n".encode())
    data = await r.read()
    w.close()
    return int(data.split(b" ", 2)[1]), data.split(b"\r\n\r\n", 1)[1]


async def _until(pred, timeout: float, what: str) -> float:
    t0 = time.monotonic()
    while True:
        if await pred():
            return time.monotonic() - t0
        assert time.monotonic() - t0 < timeout, what
        await asyncio.sleep(0.05)


def test_healthz_goes_503_when_a_shard_queue_is_deleted_and_back_to_200(tmp_path):
    """An operator deletes shard queue v1.download-1, which belongs to someone
    else (quorum, so the worker may not re-declare it): its consumer is
    cancelled and every re-subscribe fails.  /healthz answers 503 within
    health_down_s (plus one probe); once the queue exists again the shard
    re-subscribes by itself and /healthz is 200 again."""
    async def main():
        port = _free_port()
        e = await Env().up(tmp_path, metrics_addr=f"127.0.0.1:{port}", health_down_s=0.5,
                           predeclare={"v1.download": {"x-queue-type": "quorum"}})
        assert (await _get(port))[0] == 200
        e.broker.delete_queue("v1.download-1")
        t = await _until(lambda: _status(port, 503), 5.0, "never went 503")
        assert t < 0.5 + 1.5, t
        code, body = await _get(port)
        assert code == 503 and b"no consumer on v1.download-1" in body, body
        code, m = await _get(port, "/metrics")
        assert b'tritondl_consumer_active{queue="v1.download-1"} 0.0' in m
        assert b'tritondl_consumer_active{queue="v1.download-0"} 1.0' in m
        e.broker.declare("v1.download", queue_args={"x-queue-type": "quorum"})
        await _until(lambda: _status(port, 200), 10.0, "never came back to 200")
        # and it consumes again
        url = e.origin.add("/h.mkv", os.urandom(5000))
        e.submit(Media(id="h1", source_uri=url), i=1)
        res = await e.wait_results(1)
        assert res[0].ok, res[0]
        await e.down()
    run(main())


async def _status(port: int, want: int) -> bool:
    try:
        return (await _get(port))[0] == want
    except OSError:
        return False


def test_healthz_503_when_the_worker_may_no_longer_read_a_shard(tmp_path):
    """Permissions revoked on one shard: the consumer is cancelled (queue
    deleted and re-created by its owner), the re-subscribe gets 403 forever."""
    async def main():
        e = await Env().up(tmp_path, user="dl", perms=dict(configure=r"^v1\.download(-\d+)?$",
                                                          write=r"^(v1\.download(-\d+)?|v1\.convert)$",
                                                          read=r"^v1\.download(-\d+)?$"),
                           health_down_s=0.3, predeclare={"v1.convert": None})
        ok, why = await e.svc.health()
        assert ok, why
        e.broker.users["dl"][1].read = r"^v1\.download(-0)?$"   # shard 1 no longer readable
        e.broker.delete_queue("v1.download-1")

        async def red():
            ok, why = await e.svc.health()
            return not ok and any("v1.download-1" in w for w in why)
        await _until(red, 5.0, "health stayed green")
        assert ("dl", "read", "queue", "v1.download-1") in e.broker.refusals
        e.broker.users["dl"][1].read = r"^v1\.download(-\d+)?$"

        async def green():
            return (await e.svc.health())[0]
        await _until(green, 10.0, "health never recovered")
        await e.down()
    run(main())


def test_healthz_503_while_the_broker_stays_down(tmp_path):
    """The supervisor keeps redialling a broker that is gone: 503 after
    health_down_s, 200 again once it is back and the shards consume."""
    async def main():
        e = await Env().up(tmp_path, health_down_s=0.4)
        port = e.broker.port
        await e.broker.stop()

        async def red():
            ok, why = await e.svc.health()
            return not ok and any("broker connection down" in w for w in why)
        await _until(red, 5.0, "health stayed green with the broker gone")
        e.svc._collect_gauges()
        assert e.svc.metrics.get("broker_down_seconds") > 0.3
        e.broker = await Broker(port=port).start()

        async def green():
            return (await e.svc.health())[0]
        await _until(green, 15.0, "health never recovered after the broker came back")
        e.svc._collect_gauges()
        assert e.svc.metrics.get("broker_down_seconds") == 0.0
        await e.down()
    run(main(), timeout=90)


def test_healthz_503_when_idle_on_a_backlog(tmp_path):
    """Consumers registered, a free job slot, ready messages piling up and
    nothing delivered (a stuck queue): 503 after health_stall_s."""
    async def main():
        e = await Env().up(tmp_path, health_stall_s=0.3)
        e.broker.pause_delivery(True)
        url = e.origin.add("/s.mkv", os.urandom(5000))
        for k in range(3):
            e.submit(Media(id=f"s{k}", source_uri=url), i=k)
        e.svc._backlog = (0.0, 0)               # do not wait out the 5 s poll cache

        async def red():
            ok, why = await e.svc.health()
            e.svc._backlog = (0.0, e.svc._backlog[1]) if ok else e.svc._backlog
            return not ok and any("ready messages" in w for w in why)
        await _until(red, 5.0, "a stalled worker looked healthy")
        e.broker.pause_delivery(False)
        await e.wait_results(3)
        e.svc._backlog = (0.0, 0)
        ok, why = await e.svc.health()
        assert ok, why
        e.svc._collect_gauges()
        assert e.svc.metrics.get("last_job_finished_age_seconds") < 1.0
        await e.down()
    run(main())


def test_metrics_collectors_run_on_render():
    m = Metrics()
    m.collectors.append(lambda: m.set("x", 7))
    assert "tritondl_x 7" in m.render()


def test_healthz_answers_at_once_while_the_backlog_poll_is_slow(tmp_path):
    """The backlog count behind the stall check is polled in the background:
    a broker slow to answer the passive declares never makes /healthz slow
    (a probe's own timeout is often 1 s)."""
    async def main():
        e = await Env().up(tmp_path, health_stall_s=0.3)

        async def slow(topic):
            await asyncio.sleep(10)
            return {}
        e.amqp.ready_counts = slow
        t0 = time.monotonic()
        for _ in range(5):
            ok, why = await e.svc.health()
            assert ok, why
        assert time.monotonic() - t0 < 0.5
        e.svc._backlog_task.cancel()
        await e.down()
    run(main())


def test_a_backlog_behind_a_full_shard_consumer_is_not_a_stall(tmp_path):
    """two job slots, one shard consumer's prefetch taken by a
    long job, a backlog on that same shard and the other shard empty.  The
    free slot cannot be given shard 0's backlog (its consumer is full), so
    the worker is not stalled and /healthz stays 200; once the long job ends
    the backlog runs."""
    async def main():
        e = await Env().up(tmp_path, health_stall_s=0.3, concurrency=2)
        e.svc._prefetch_for = lambda limit: 1          # the case the advice describes: prefetch 1 per shard
        await e.amqp.set_live_prefetch(1)
        e.origin.rate = 1_000_000
        long_url = e.origin.add("/long.mkv", os.urandom(2_500_000))
        short_url = e.origin.add("/short.mkv", os.urandom(5000))
        e.submit(Media(id="long", source_uri=long_url), i=0)
        t0 = time.monotonic()
        while not any(r[1] == "/long.mkv" for r in e.origin.requests):
            assert time.monotonic() - t0 < 5
            await asyncio.sleep(0.01)
        for k in range(3):
            e.submit(Media(id=f"b{k}", source_uri=short_url), i=0)      # same shard as the long job
        assert not e.amqp.shards["v1.download-0"].has_room(1) and e.amqp.shards["v1.download-1"].has_room(1)
        t1 = time.monotonic()
        while time.monotonic() - t1 < 1.2:
            e.svc._backlog = (0.0, e.svc._backlog[1])  # re-poll on every probe
            ok, why = await e.svc.health()
            assert ok, why
            await asyncio.sleep(0.1)
        assert e.svc._backlog[1] == 0                  # shard 0's ready messages were not counted
        res = await e.wait_results(4, timeout=30)
        assert all(r.ok for r in res), res
        await e.down()
    run(main())
