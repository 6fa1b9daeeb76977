"""RabbitMQ's consumer_timeout (3.8.15+; 30 min by default): a delivery left
unacked longer than that closes its channel with 406 PRECONDITION_FAILED and
goes back to the queue.  A long job (a multi-GB torrent behind a 10-minute
metadata wait) does exactly that in production, as it would have with the
reference (which held the delivery unacked for the whole job,
``cmd/downloader/downloader.go:103-155``).  The worker must say so clearly,
get its shard consuming again, and not run the job a second time when the
broker redelivers it."""

import asyncio
import os

from tritondl.models import Media
from tritondl.s3.uploader import object_key

from .test_permissions import Env, run


def test_fake_broker_closes_a_channel_holding_a_delivery_past_the_timeout():
    from tritondl.amqp import codec
    from tritondl.amqp.connection import ChannelClosed, Connection
    from tritondl_testkit.fakes.broker import Broker

    async def main():
        b = await Broker().start()
        b.consumer_timeout = 0.2
        b.declare("t")
        conn = await Connection.open(b.url, heartbeat=0)
        ch = await conn.channel()
        got = []
        closed = asyncio.get_running_loop().create_future()
        ch.add_close_callback(lambda e: closed.done() or closed.set_result(e))
        await ch.basic_consume("t-0", got.append)
        b.inject("t", "t-0", b"job")
        err = await asyncio.wait_for(closed, 5)
        assert isinstance(err, ChannelClosed) and err.code == codec.PRECONDITION_FAILED
        assert "delivery acknowledgement on channel" in str(err) and "timed out" in str(err)
        assert len(got) == 1 and b.queue_depth("t-0") == 1          # requeued
        assert b.queues["t-0"].messages[0].redelivered
        await conn.close()
        await b.stop()
    run(main())


def test_job_longer_than_the_consumer_timeout_runs_once(tmp_path):
    """The job outlives the broker's consumer timeout: its channel is closed
    under it and the delivery requeued.  The job still finishes (upload +
    v1.convert), the shard consumes again, and the redelivered copy is acked
    without a second download or a second v1.convert."""
    async def main():
        e = await Env().up(tmp_path, health_down_s=0.5)
        e.broker.consumer_timeout = 0.3
        data = os.urandom(3 << 20)
        url = e.origin.add("/long.mkv", data)
        e.origin.rate = 3_000_000                        # 1 MiB steps, ~0.35 s apart: past the timeout
        e.submit(Media(id="long", source_uri=url))
        res = await e.wait_results(2, timeout=20)
        assert [r.stage for r in res] == ["done", "duplicate"], res
        assert e.s3.object_bytes("triton-staging", object_key("long", "long.mkv")) == data
        gets = [r for r in e.origin.requests if r[0] == "GET" and r[1] == "/long.mkv"]
        await asyncio.sleep(0.3)
        assert [c.media.id for c in e.converts()] == ["long"]       # one v1.convert
        assert [r for r in e.origin.requests if r[0] == "GET" and r[1] == "/long.mkv"] == gets
        assert e.broker.stats["consumer_timeouts"] >= 1 and e.amqp.consumer_timeouts >= 1
        assert e.svc.metrics.get("jobs", status="duplicate") == 1
        assert e.broker.unacked_count() == 0 and e.broker.queue_depth("v1.download-0") == 0
        ok, why = await e.svc.health()
        assert ok, why                                    # the shard is consuming again
        await e.down()
    run(main())
