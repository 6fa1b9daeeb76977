"""AMQP layer: codec, connection ↔ fake broker, and the job client
(topology, fan-in, round-robin publish, X-Retries, reconnect)."""

import asyncio
from decimal import Decimal

import pytest

from tritondl.amqp import codec
from tritondl.amqp.client import Client, _parse_retries
from tritondl.amqp.codec import Method, Properties
from tritondl.amqp.connection import ChannelClosed, Connection, ConnectionClosed, PublishNacked, parse_url
from tritondl_testkit.fakes.broker import Broker
from tritondl.utils.backoff import ExponentialBackoff


def run(coro, timeout=20):
    return asyncio.run(asyncio.wait_for(coro, timeout))


# ------------------------------------------------------------------ codec


def test_table_roundtrip():
    t = {"a": 1, "b": "str", "c": True, "d": 2**40, "e": 1.5, "f": {"x": [1, "y", None]}, "g": b"\x00\x01",
         "h": Decimal("1.25")}
    assert codec.decode_table(codec.encode_table(t)) == t


def test_method_roundtrip_with_bits():
    m = Method("queue.declare", {"queue": "q", "passive": False, "durable": True, "exclusive": False,
                                 "auto_delete": True, "nowait": False, "arguments": {"x-max": 5}})
    d = codec.decode_method(codec.encode_method(m))
    assert d.name == "queue.declare" and d.durable and d.auto_delete and not d.exclusive
    assert d.arguments == {"x-max": 5}
    # bit packing: 5 consecutive bits -> one octet
    raw = codec.encode_method(m)
    assert raw.endswith(codec.encode_table({"x-max": 5}))


def test_header_roundtrip():
    p = Properties(content_type="application/octet-stream", delivery_mode=2, headers={"X-Retries": 3},
                   message_id="m1", timestamp=123)
    cid, size, q = codec.decode_header(codec.encode_header(60, 99, p))
    assert (cid, size) == (60, 99) and q == p


def test_parse_url():
    p = parse_url("amqp://u%40x:p%2F@h:1234/v%2Fh")
    assert (p.username, p.password, p.host, p.port, p.vhost) == ("u@x", "p/", "h", 1234, "v/h")
    p = parse_url("amqp://:@127.0.0.1:5672")
    assert p.vhost == "/" and p.username == ""


def test_parse_retries():
    assert _parse_retries(None) == 0
    assert _parse_retries({"X-Retries": 4}) == 4
    assert _parse_retries({"X-Retries": "4"}) == 0
    assert _parse_retries({"X-Retries": 2**40}) == 0


# ------------------------------------------------------- connection/broker


def test_publish_consume_ack_and_prefetch():
    async def main():
        b = await Broker().start()
        conn = await Connection.open(b.url)
        ch = await conn.channel()
        await ch.exchange_declare("ex", "direct", durable=True)
        await ch.queue_declare("q", durable=True)
        await ch.queue_bind("q", "ex", "q")
        await ch.confirm_select()
        for i in range(5):
            await ch.basic_publish("ex", "q", f"m{i}".encode(), Properties(delivery_mode=2))
        cch = await conn.channel()
        await cch.basic_qos(2, 0, True)
        got = []
        await cch.basic_consume("q", got.append)
        await asyncio.sleep(0.05)
        assert [m.body for m in got] == [b"m0", b"m1"]  # prefetch 2, nothing acked yet
        await got[0].ack()
        await asyncio.sleep(0.05)
        assert len(got) == 3
        await got[1].nack(requeue=True)
        await asyncio.sleep(0.05)
        assert got[-1].body == b"m1" and got[-1].redelivered
        # large body is split over frames
        big = bytes(range(256)) * 4000
        await ch.basic_publish("ex", "q", big)
        acked = 1
        for _ in range(50):
            for m in got[acked:]:
                if m.body != b"m1" or m.redelivered:
                    await m.ack()
            acked = len(got)
            await asyncio.sleep(0.02)
            if any(m.body == big for m in got):
                break
        assert any(m.body == big for m in got)
        await conn.close()
        await b.stop()
    run(main())


def test_close_requeues_unacked_and_channel_errors():
    async def main():
        b = await Broker().start()
        c1 = await Connection.open(b.url)
        ch = await c1.channel()
        await ch.queue_declare("q")
        await ch.basic_publish("", "q", b"job")
        got = []
        await ch.basic_consume("q", got.append)
        await asyncio.sleep(0.05)
        assert len(got) == 1 and not got[0].redelivered
        await c1.close()
        c2 = await Connection.open(b.url)
        ch2 = await c2.channel()
        got2 = []
        await ch2.basic_consume("q", got2.append)
        await asyncio.sleep(0.05)
        assert got2[0].body == b"job" and got2[0].redelivered
        # inequivalent redeclare -> channel closed 406, connection survives
        with pytest.raises(ChannelClosed) as ei:
            await ch2.queue_declare("q", durable=True)
        assert ei.value.code == codec.PRECONDITION_FAILED
        ch3 = await c2.channel()
        with pytest.raises(ChannelClosed) as ei:
            await ch3.queue_declare("nope", passive=True)
        assert ei.value.code == codec.NOT_FOUND
        assert not c2.is_closed
        await c2.close()
        await b.stop()
    run(main())


def test_confirms_nack_injection_and_dead_letter():
    async def main():
        b = await Broker().start()
        conn = await Connection.open(b.url)
        ch = await conn.channel()
        await ch.exchange_declare("dlx", "fanout")
        await ch.queue_declare("dead")
        await ch.queue_bind("dead", "dlx")
        await ch.queue_declare("work", arguments={"x-dead-letter-exchange": "dlx"})
        await ch.confirm_select()
        b.fail_next_publishes(1)
        with pytest.raises(PublishNacked):
            await ch.basic_publish("", "work", b"x")
        await ch.basic_publish("", "work", b"y")
        m = await ch.basic_get("work")
        assert m.body == b"y"
        await m.nack(requeue=False)
        await asyncio.sleep(0.02)
        assert b.queue_depth("dead") == 1
        assert b.drain_queue("dead")[0].props.headers["x-death"][0]["queue"] == "work"
        assert await ch.basic_get("work") is None
        await conn.close()
        await b.stop()
    run(main())


def test_auth_refused_and_blocked():
    async def main():
        b = await Broker(username="u", password="p").start()
        with pytest.raises(ConnectionClosed):
            await Connection.open(f"amqp://u:wrong@{b.endpoint}/")
        conn = await Connection.open(f"amqp://u:p@{b.endpoint}/")
        ch = await conn.channel()
        await ch.queue_declare("q")
        b.set_blocked(True)
        await asyncio.sleep(0.02)
        t = asyncio.ensure_future(ch.basic_publish("", "q", b"z"))
        await asyncio.sleep(0.05)
        assert not t.done()
        b.set_blocked(False)
        await asyncio.wait_for(t, 2)
        await asyncio.sleep(0.05)
        assert b.queue_depth("q") == 1
        await conn.close()
        await b.stop()
    run(main())


def test_heartbeat_detects_dead_peer():
    async def main():
        # a "server" that completes the handshake and then goes silent
        b = await Broker(heartbeat=1).start()
        conn = await Connection.open(b.url, heartbeat=1)
        for c in list(b.conns):  # stop reading/writing on the server side
            c.closed = True
        err = await asyncio.wait_for(conn.wait_closed(), 5)
        assert "heartbeat" in str(err) or isinstance(err, ConnectionClosed)
        await b.stop()
    run(main())


# ------------------------------------------------------------------ client


def test_client_topology_fanin_and_round_robin():
    async def main():
        b = await Broker().start()
        cl = await Client(b.url, prefetch=1).connect()
        stream = await cl.consume("v1.download")
        assert {"v1.download-0", "v1.download-1"} <= set(b.queues)
        ex = b.exchanges["v1.download"]
        assert ex.type == "direct" and ex.durable
        assert sorted(x[:2] for x in ex.bindings) == [("v1.download-0", "v1.download-0"),
                                                       ("v1.download-1", "v1.download-1")]
        for i in range(4):
            await cl.publish("v1.download", f"j{i}".encode())
        rks = [m.routing_key for m in b.published]
        assert rks == ["v1.download-0", "v1.download-1"] * 2
        assert all(m.props.delivery_mode == 2 and m.props.content_type == "application/octet-stream"
                   for m in b.published)
        seen = []
        async for d in stream:
            seen.append(d.body)
            await d.ack()
            if len(seen) == 4:
                break
        assert sorted(seen) == [b"j0", b"j1", b"j2", b"j3"]
        await cl.close()
        await b.stop()
    run(main())


def test_client_retry_increments_x_retries():
    async def main():
        b = await Broker().start()
        cl = await Client(b.url, prefetch=1, retry_delay=0).connect()
        await cl.consume("t")
        await cl.publish("t", b"job")
        d = await cl.get(2)
        assert d.metadata.retries == 0
        await d.retry()
        d2 = await cl.get(2)
        assert d2.body == b"job" and d2.metadata.retries == 1 and d2.routing_key == d.routing_key
        await d2.nack()
        await asyncio.sleep(0.05)
        assert b.queue_depth("t-0") + b.queue_depth("t-1") == 0
        await cl.close()
        await b.stop()
    run(main())


def test_client_reconnects_and_redelivers():
    async def main():
        b = await Broker().start()
        cl = Client(b.url, prefetch=1, heartbeat=0,
                    backoff=ExponentialBackoff(initial=0.02, max_interval=0.1, max_elapsed=10))
        await cl.connect()
        await cl.consume("t")
        await cl.publish("t", b"a")
        d = await cl.get(2)
        assert d.body == b"a" and not d.redelivered
        await b.drop_connections()
        for _ in range(100):
            if cl.reconnects and cl.connected:
                break
            await asyncio.sleep(0.02)
        assert cl.reconnects == 1
        await d.ack()  # stale: must not raise
        d2 = await cl.get(3)
        assert d2.body == b"a" and d2.redelivered
        await d2.ack()
        await cl.publish("t", b"b")  # publisher channel re-created on the new connection
        d3 = await cl.get(2)
        assert d3.body == b"b"
        await d3.ack()
        await cl.close()
        await b.stop()
    run(main())


def test_client_publish_retries_after_nack():
    async def main():
        b = await Broker().start()
        cl = await Client(b.url).connect()
        b.fail_next_publishes(2)
        await cl.publish("v1.convert", b"c")
        assert b.queue_depth("v1.convert-0") == 1
        await cl.close()
        await b.stop()
    run(main())


def test_client_resubscribes_after_server_cancel():
    """A queue deleted under a consumer (or a failover) makes the broker send
    basic.cancel; the client re-declares the shard queue and consumes again."""
    async def main():
        b = await Broker().start()
        cl = await Client(b.url, prefetch=1).connect()
        stream = await cl.consume("v1.download")
        admin = await Connection.open(b.url, heartbeat=0)
        ach = await admin.channel()
        await ach.queue_delete("v1.download-1")
        for _ in range(100):
            q = b.queues.get("v1.download-1")
            if q is not None and q.consumers:
                break
            await asyncio.sleep(0.02)
        assert b.queues["v1.download-1"].consumers          # resubscribed
        await cl.publish("v1.download", b"a")               # -> v1.download-0
        await cl.publish("v1.download", b"b")               # -> v1.download-1 (the re-created queue)
        got = []
        async for d in stream:
            got.append(d.body)
            await d.ack()
            if len(got) == 2:
                break
        assert sorted(got) == [b"a", b"b"]
        await admin.close()
        await cl.close()
        await b.stop()
    run(main())


def test_client_reopens_consumer_channel_closed_by_broker():
    """A 406 (unknown delivery tag) closes a consumer channel on the broker;
    the client opens a new one and keeps consuming that shard."""
    async def main():
        b = await Broker().start()
        cl = await Client(b.url, prefetch=1).connect()
        stream = await cl.consume("v1.download")
        victim = cl._consumer_chans[0]
        victim.conn._send_method(victim.id, Method("basic.ack", {"delivery_tag": 9999, "multiple": False}))
        for _ in range(100):
            if victim.is_closed and len(b.queues["v1.download-0"].consumers) == 1 and \
                    len(cl._consumer_chans) == 2:
                break
            await asyncio.sleep(0.02)
        assert victim.is_closed and len(cl._consumer_chans) == 2
        for i in range(4):
            await cl.publish("v1.download", f"m{i}".encode())
        got = []
        async for d in stream:
            got.append(d.body)
            await d.ack()
            if len(got) == 4:
                break
        assert sorted(got) == [b"m0", b"m1", b"m2", b"m3"]
        await cl.close()
        await b.stop()
    run(main())


def test_fast_method_codecs_match_the_generic_path():
    """The hand-packed basic.ack/nack/deliver/publish encoders and decoders
    produce exactly what the table-driven codec does (random arguments,
    bit combinations, unicode short strings)."""
    import random
    from tritondl.amqp import codec as cd

    def generic_encode(m):
        f = cd._FAST_ENC.pop(m.name)
        try:
            return cd.encode_method(m)
        finally:
            cd._FAST_ENC[m.name] = f

    def generic_decode(b):
        r = cd._Reader(b)
        cid, mid = r.unpack(">HH")
        name, args = cd.METHODS[(cid, mid)]
        return cd.Method(name, {a: getattr(r, t)() for a, t in args})

    rng = random.Random(5)
    words = ["", "v1.download", "v1.download-1", "amq.ctag-é" * 3, "x" * 255]
    for _ in range(400):
        tag = rng.choice([0, 1, 2 ** 63 - 1, rng.randrange(2 ** 64)])
        b1, b2 = rng.random() < 0.5, rng.random() < 0.5
        for m in (cd.Method("basic.ack", {"delivery_tag": tag, "multiple": b1}),
                  cd.Method("basic.nack", {"delivery_tag": tag, "multiple": b1, "requeue": b2}),
                  cd.Method("basic.deliver", {"consumer_tag": rng.choice(words), "delivery_tag": tag,
                                              "redelivered": b1, "exchange": rng.choice(words),
                                              "routing_key": rng.choice(words)}),
                  cd.Method("basic.publish", {"ticket": rng.randrange(65536), "exchange": rng.choice(words),
                                              "routing_key": rng.choice(words), "mandatory": b1, "immediate": b2})):
            raw = cd.encode_method(m)
            assert raw == generic_encode(m)
            assert cd.decode_method(raw) == generic_decode(raw) == m
    # defaults (missing args) encode like the generic path
    for name in ("basic.ack", "basic.nack", "basic.deliver", "basic.publish"):
        assert cd.encode_method(cd.Method(name, {})) == generic_encode(cd.Method(name, {}))
    # malformed hot-method payloads still raise the codec's FrameError
    with pytest.raises(cd.FrameError):
        cd.decode_method(bytes.fromhex("003c003c05"))


def test_fake_broker_heartbeats_both_ways():
    """The fake broker sends heartbeats on a silent connection and drops a
    peer that stopped sending them (RabbitMQ), so idle heartbeating clients
    survive and dead ones are detected on both ends."""
    import asyncio as aio

    from tritondl.amqp.connection import Connection
    from tritondl_testkit.fakes.broker import Broker

    async def main():
        b = await Broker(heartbeat=1).start()
        c = await Connection.open(b.url, heartbeat=1)
        await aio.sleep(3.0)                               # idle: only heartbeats flow
        assert not c.is_closed and len(b.conns) == 1
        assert b.stats["heartbeats_sent"] >= 3
        for t in list(c._tasks):                           # the client goes silent (a hung peer)
            t.cancel()
        for _ in range(60):
            if not b.conns:
                break
            await aio.sleep(0.1)
        assert not b.conns and b.stats["heartbeat_timeouts"] == 1
        await b.stop()
    aio.run(aio.wait_for(main(), 30))


def test_channel_housekeeping_methods():
    """The rest of the channel surface against the fake broker: purge,
    cancel, recover, unbind and exchange delete behave as RabbitMQ's."""
    async def main():
        b = await Broker().start()
        conn = await Connection.open(b.url)
        ch = await conn.channel()
        await ch.exchange_declare("hk", "direct", durable=True)
        await ch.queue_declare("hk-q", durable=True)
        await ch.queue_bind("hk-q", "hk", "hk-q")
        await ch.confirm_select()
        for i in range(3):
            await ch.basic_publish("hk", "hk-q", b"x%d" % i)
        assert await ch.queue_purge("hk-q") == 3
        assert b.queue_depth("hk-q") == 0
        # a cancelled consumer gets nothing more; recover hands its unacked delivery back
        cch = await conn.channel()
        got = []
        tag = await cch.basic_consume("hk-q", got.append)
        await ch.basic_publish("hk", "hk-q", b"first")
        for _ in range(50):
            if got:
                break
            await asyncio.sleep(0.01)
        await cch.basic_cancel(tag)
        await ch.basic_publish("hk", "hk-q", b"second")
        await asyncio.sleep(0.05)
        assert [m.body for m in got] == [b"first"]
        await cch.basic_recover(requeue=True)
        for _ in range(50):
            if b.queue_depth("hk-q") == 2:
                break
            await asyncio.sleep(0.01)
        assert b.queue_depth("hk-q") == 2
        # unbound: the routing key no longer reaches the queue
        await ch.queue_unbind("hk-q", "hk", "hk-q")
        await ch.basic_publish("hk", "hk-q", b"dropped")
        assert b.queue_depth("hk-q") == 2
        await ch.exchange_delete("hk")
        with pytest.raises(ChannelClosed) as e:
            await ch.exchange_declare("hk", "direct", passive=True)
        assert e.value.code == codec.NOT_FOUND
        await conn.close()
        await b.stop()
    run(main())


def test_mandatory_publish_surfaces_unroutable_messages():
    """RabbitMQ confirms a message no queue is bound for and drops it.  With
    ``mandatory`` it sends ``basic.return`` first; the channel matches the
    return to its publish by a private ``x-tdl-seq`` header, not the
    producer's message_id (an unroutable message is confirmed
    at once, ahead of routable ones still being persisted, so order cannot
    match them) and fails that publish's confirm with PublishReturned."""
    from tritondl.amqp.connection import PublishReturned

    async def main():
        b = await Broker().start()
        conn = await Connection.open(b.url)
        ch = await conn.channel()
        await ch.exchange_declare("ex", "direct", durable=True)
        await ch.queue_declare("bound", durable=True)
        await ch.queue_bind("bound", "ex", "bound")
        await ch.confirm_select()
        futs = [await ch.basic_publish("ex", rk, b"m", Properties(delivery_mode=2), mandatory=True,
                                       wait_confirm=False) for rk in ("bound", "nowhere", "bound", "nowhere")]
        res = await asyncio.gather(*futs, return_exceptions=True)
        assert res[0] is True and res[2] is True
        assert isinstance(res[1], PublishReturned) and isinstance(res[3], PublishReturned)
        assert res[1].code == codec.NO_ROUTE and res[1].routing_key == "nowhere"
        assert b.queue_depth("bound") == 2
        # a caller's own message_id is left alone, and two publishes in flight may share it:
        # the return is charged to the unroutable one only
        with pytest.raises(PublishReturned):
            await ch.basic_publish("ex", "nowhere", b"m", Properties(message_id="job-42"), mandatory=True)
        f1 = await ch.basic_publish("ex", "bound", b"a", Properties(message_id="job-42"), mandatory=True,
                                    wait_confirm=False)
        f2 = await ch.basic_publish("ex", "nowhere", b"b", Properties(message_id="job-42"), mandatory=True,
                                    wait_confirm=False)
        r = await asyncio.gather(f1, f2, return_exceptions=True)
        assert r[0] is True and isinstance(r[1], PublishReturned), r
        assert b.queues["bound"].messages[-1].props.message_id == "job-42"
        assert b.queues["bound"].messages[-1].body == b"a"
        assert not ch._mandatory_ids and not ch._returned
        # without mandatory the broker drops it and confirms (the reference's publish)
        await ch.basic_publish("ex", "nowhere", b"m")
        await conn.close()
        await b.stop()
    run(main())


def test_client_redeclares_a_deleted_publish_queue_instead_of_losing_the_message():
    """An operator deletes a v1.convert shard queue under a running worker:
    the next publish to it comes back unroutable; the client forgets its
    declared-topology cache, declares the queue and binding again and
    publishes, so the message lands instead of vanishing."""
    async def main():
        b = await Broker().start()
        cl = await Client(b.url, prefetch=1).connect()
        await cl.publish("v1.convert", b"first")
        await cl.publish("v1.convert", b"second")
        assert b.queue_depth("v1.convert-0") == 1 and b.queue_depth("v1.convert-1") == 1
        b.delete_queue("v1.convert-0")
        await cl.publish("v1.convert", b"third")          # round robin: shard 0, now gone
        assert cl.returned == 1
        assert [m.body for m in b.drain_queue("v1.convert-0")] == [b"third"]
        await cl.close()
        await b.stop()
    run(main())


def test_unroutable_publish_on_foreign_topology_fails_after_retries():
    """A topology the worker may not declare (write-only user) that has no
    queue for a routing key: the publish is retried, then fails loudly, so
    the job is not acked as if its result had been delivered."""
    from tritondl.amqp.connection import PublishReturned

    async def main():
        b = await Broker().start()
        b.add_user("w", "w", configure="^$", write=".*", read=".*")
        b.declare("v1.convert", 1)                        # only v1.convert-0 exists
        cl = await Client(b.url.replace("guest:guest", "w:w"), prefetch=1).connect()
        await cl.publish("v1.convert", b"ok", max_attempts=3)
        with pytest.raises(PublishReturned):
            await cl.publish("v1.convert", b"lost?", max_attempts=3)
        assert cl.returned == 3 and "v1.convert" in cl.external_topics
        assert b.queue_depth("v1.convert-0") == 1
        await cl.close()
        await b.stop()
    run(main())


def test_deleted_delay_queue_is_declared_again_not_lost():
    """The retry copy goes to a delay queue through the default exchange; if
    the queue was deleted after it was declared, the copy would be dropped
    and the original acked.  The return makes the client declare it again."""
    async def main():
        b = await Broker().start()
        cl = await Client(b.url, prefetch=1, retry_delay=5).connect()
        await cl.consume("t")
        names = [cl.delay_queue_name(f"t-{i}", 5) for i in range(2)]
        for body in (b"j0", b"j1"):                       # one per shard: both delay queues declared
            await cl.publish("t", body)
            await (await cl.get(2)).retry(5)
        assert [b.queue_depth(n) for n in names] == [1, 1]
        for n in names:
            b.delete_queue(n)
        await cl.publish("t", b"j2")
        d = await cl.get(2)
        await d.retry(5)
        name = cl.delay_queue_name(d.routing_key, 5)
        assert b.queue_depth(name) == 1 and b.drain_queue(name)[0].body == b"j2"
        await cl.close()
        await b.stop()
    run(main())


def test_client_redeclares_a_deleted_publish_exchange():
    """The v1.convert exchange is deleted under a running worker: the publish
    is a 404 channel error; the client forgets it ever declared the topic,
    declares it again on the retry, and the message lands."""
    async def main():
        b = await Broker().start()
        cl = await Client(b.url, prefetch=1).connect()
        await cl.publish("v1.convert", b"first")
        assert b.delete_exchange("v1.convert")
        await cl.publish("v1.convert", b"second", max_attempts=4)
        assert "v1.convert" in b.exchanges
        got = [m.body for q in ("v1.convert-0", "v1.convert-1") for m in b.drain_queue(q)]
        assert sorted(got) == [b"first", b"second"]
        await cl.close()
        await b.stop()
    run(main())


def test_connection_names_its_worker_process():
    """client_properties.connection_name: the management UI shows which
    worker process on which host holds a connection."""
    import os
    import socket

    async def main():
        b = await Broker().start()
        conn = await Connection.open(b.url)
        props = next(iter(b.conns)).client_properties
        name = props["connection_name"]
        name = name.decode() if isinstance(name, bytes) else name
        assert name == f"tritondl@{socket.gethostname()} pid {os.getpid()}"
        assert props["capabilities"]["publisher_confirms"] is True
        await conn.close()
        await b.stop()
    run(main())


def test_pause_hands_buffered_deliveries_back_and_resume_consumes_again():
    """A worker busy with a long job holds one more delivery per other shard.
    pause() cancels the consumers, re-publishes the buffered delivery (a
    fresh message: not marked redelivered) and acks the original; while
    paused nothing more arrives and health stays green; resume() consumes."""
    async def main():
        b = await Broker().start()
        cl = await Client(b.url, prefetch=1).connect()
        await cl.consume("t")
        await cl.publish("t", b"long")                 # shard 0
        await cl.publish("t", b"waiting")              # shard 1: buffered behind the long job
        running = await cl.get(2)
        for _ in range(50):
            if not cl._out.empty():
                break
            await asyncio.sleep(0.01)
        assert not cl._out.empty()
        assert await cl.pause() == 1 and cl.paused and cl.handed_back == 1
        assert all(not sh.active and sh.paused for sh in cl.shards.values())
        assert cl.health(0.0) == (True, [])
        other = "t-1" if running.routing_key == "t-0" else "t-0"
        back = b.queues[other].messages
        assert len(back) == 1 and back[0].body == b"waiting" and not back[0].redelivered
        await cl.publish("t", b"later")
        await asyncio.sleep(0.1)
        assert cl._out.empty()                         # paused: nothing delivered
        assert await cl.pause() == 0                   # idempotent
        await running.ack()                            # acks still work on the paused channel
        await cl.resume()
        assert not cl.paused and all(sh.active for sh in cl.shards.values())
        got = sorted([(await cl.get(2)).body, (await cl.get(2)).body])
        assert got == [b"later", b"waiting"]
        await cl.close()
        await b.stop()
    run(main())


def test_a_redelivered_delivery_handed_back_stays_a_possible_duplicate():
    """pause() re-publishes buffered deliveries as fresh messages.  One the
    broker had flagged redelivered (an ack that went nowhere) keeps being
    checked against the done-ledger: its copy carries X-Tdl-Redelivered.
    A retry of it drops the mark."""
    from tritondl.amqp.client import REDELIVERED

    async def main():
        b = await Broker().start()
        cl = await Client(b.url, prefetch=1).connect()
        await cl.consume("t")
        b.inject("t", "t-0", b"long", Properties(delivery_mode=2))
        running = await cl.get(2)
        assert running.body == b"long"
        b.pause_delivery(True)
        b.inject("t", "t-1", b"dup", Properties(delivery_mode=2, headers={"X-Retries": 1}))
        b.queues["t-1"].messages[-1].redelivered = True
        b.pause_delivery(False)
        for _ in range(50):
            if not cl._out.empty():
                break
            await asyncio.sleep(0.01)
        assert await cl.pause() == 1
        back = b.queues["t-1"].messages
        assert len(back) == 1 and not back[0].redelivered
        assert back[0].props.headers[REDELIVERED] == 1 and back[0].props.headers["X-Retries"] == 1
        await running.ack()
        await cl.resume()
        d = await cl.get(2)
        assert d.body == b"dup" and not d.redelivered and d.maybe_duplicate
        assert REDELIVERED not in d.retry_props().headers
        await d.ack()
        await cl.close()
        await b.stop()
    run(main())
