"""In-process AMQP 0-9-1 broker (asyncio, TCP) — the RabbitMQ stand-in for
tests, the smoke check and bench.py.  The reference had no fake broker at all
(zero coverage of the messaging layer).

Implements the RabbitMQ semantics the worker depends on:

* PLAIN auth, tune/open, heartbeats, channel open/close/flow;
* direct / fanout / topic exchanges plus the default exchange; durable /
  argument equivalence checks (406 PRECONDITION_FAILED on mismatch);
* queues with round-robin consumers, ``basic.qos`` prefetch (RabbitMQ
  reading: ``global=true`` → per-channel limit, ``false`` → per-consumer,
  captured when the consumer starts: a later ``basic.qos`` only applies to
  consumers started after it).  Quorum and stream queues refuse a consumer
  on a channel with global QoS, as RabbitMQ does (540 NOT_IMPLEMENTED, a
  connection error); a stream also needs a per-consumer prefetch (406);
* manual ack/nack/reject (+``multiple``), requeue with ``redelivered``;
  unacked messages requeued when a channel or connection closes;
* dead-lettering via ``x-dead-letter-exchange`` / ``-routing-key`` on
  reject/nack and on expiry (queue ``x-message-ttl`` and per-message
  ``expiration``, expired at the queue head like RabbitMQ) — the delayed
  retry queues of :mod:`tritondl.amqp.client` are built on that;
* ``basic.get``, ``basic.cancel``, publisher confirms, ``mandatory`` returns;
* per-user permissions (:meth:`add_user`): RabbitMQ's configure / write /
  read regexes per resource, checked where RabbitMQ checks them
  (``rabbit_channel``): declare/delete need *configure* on the entity,
  publish needs *write* on the exchange (``amq.default`` for ""), bind needs
  *write* on the queue and *read* on the exchange, consume/get/purge need
  *read* on the queue, and a queue with ``x-dead-letter-exchange`` needs
  *write* on that exchange.  A refusal is a 403 channel error;
* fault injection: :meth:`drop_connections`, :meth:`set_blocked`,
  :meth:`fail_next_publishes` (nack), accept-delay.
"""

from __future__ import annotations

import asyncio
import collections
import itertools
import re
import time
from dataclasses import dataclass, field
from typing import Any

from tritondl.amqp import codec
from tritondl.amqp.codec import Method, Properties


@dataclass
class QMsg:
    body: bytes
    props: Properties
    exchange: str
    routing_key: str
    redelivered: bool = False
    expires_at: float | None = None     # monotonic deadline (queue / message TTL)


@dataclass
class Exchange:
    name: str
    type: str
    durable: bool
    auto_delete: bool = False
    internal: bool = False
    arguments: dict = field(default_factory=dict)
    bindings: list[tuple[str, str, dict]] = field(default_factory=list)  # (queue, rk, args)


@dataclass
class Queue:
    name: str
    durable: bool
    exclusive: bool = False
    auto_delete: bool = False
    arguments: dict = field(default_factory=dict)
    messages: collections.deque = field(default_factory=collections.deque)
    consumers: list = field(default_factory=list)  # [_Consumer]
    rr: int = 0
    owner: Any = None
    delivered_total: int = 0
    last_used: float = field(default_factory=time.monotonic)   # x-expires: declare, consume, get


@dataclass
class Perms:
    """One user's RabbitMQ permissions in the (single) vhost: a regex per
    access kind, matched with search semantics like RabbitMQ's ``re:run``;
    "" matches nothing (RabbitMQ stores it as ``^$``)."""
    configure: str = ".*"
    write: str = ".*"
    read: str = ".*"

    def allows(self, kind: str, name: str) -> bool:
        pat = getattr(self, kind)
        return pat != "" and re.search(pat, name) is not None


class _Consumer:
    def __init__(self, ch: "_ServerChannel", tag: str, queue: Queue, no_ack: bool, prefetch: int) -> None:
        self.ch = ch
        self.tag = tag
        self.queue = queue
        self.no_ack = no_ack
        self.prefetch = prefetch
        self.unacked = 0


class ChannelError(Exception):
    def __init__(self, code: int, text: str, cm: tuple[int, int] = (0, 0)) -> None:
        super().__init__(text)
        self.code, self.text, self.cm = code, text, cm


class ConnError(ChannelError):
    pass


def _topic_match(pattern: str, key: str) -> bool:
    """AMQP topic match: ``*`` = exactly one word, ``#`` = zero or more words."""
    pw, kw = pattern.split("."), key.split(".")

    def m(i: int, j: int) -> bool:
        if i == len(pw):
            return j == len(kw)
        if pw[i] == "#":
            return any(m(i + 1, k) for k in range(j, len(kw) + 1))
        if j == len(kw):
            return False
        return (pw[i] == "*" or pw[i] == kw[j]) and m(i + 1, j + 1)

    return m(0, 0)


class _ServerChannel:
    def __init__(self, conn: "_ServerConn", cid: int) -> None:
        self.conn = conn
        self.id = cid
        self.prefetch_channel = 0      # global=true
        self.prefetch_consumer = 0     # global=false (applies to new consumers)
        self.unacked: dict[int, tuple[QMsg, Queue, _Consumer | None]] = {}
        self.delivered_at: dict[int, float] = {}       # delivery tag -> monotonic time (consumer timeout)
        self.tags = itertools.count(1)
        self.consumers: dict[str, _Consumer] = {}
        self.confirm = False
        self.pub_seq = 0
        self.pending: tuple[Method, Properties | None, int, list[bytes]] | None = None
        self.flow = True

    def channel_unacked(self) -> int:
        return len(self.unacked)


class _ServerConn:
    def __init__(self, broker: "Broker", reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        self.broker = broker
        self.reader = reader
        self.writer = writer
        self.channels: dict[int, _ServerChannel] = {}
        self.frame_max = codec.DEFAULT_FRAME_MAX
        self.open = False
        self.closed = False
        self.client_properties: dict = {}
        self.user = ""
        self.perms: Perms | None = None            # None: every resource allowed
        self.hb = 0                                # negotiated heartbeat (s), from tune_ok
        self.last_read = time.monotonic()
        self.last_write = time.monotonic()
        self.hb_task: asyncio.Task | None = None
        self._wbuf: list[bytes] = []
        self._flush_scheduled = False
        self._delayed: collections.deque = collections.deque()   # (due, bytes) under an emulated RTT

    def send(self, data: bytes) -> None:
        """Corked: frames queued in one loop iteration go out in one write."""
        if not self.closed and not self.writer.is_closing():
            self._wbuf.append(data)
            if not self._flush_scheduled:
                self._flush_scheduled = True
                asyncio.get_running_loop().call_soon(self.flush)

    def flush(self) -> None:
        self._flush_scheduled = False
        if self._wbuf:
            data = self._wbuf[0] if len(self._wbuf) == 1 else b"".join(self._wbuf)
            self._wbuf.clear()
            rtt = self.broker.rtt
            if rtt and not self.closed:
                # emulated network: what the broker sends arrives one RTT later, in order
                self._delayed.append((time.monotonic() + rtt, data))
                if len(self._delayed) == 1:
                    asyncio.get_running_loop().call_later(rtt, self._release)
                return
            if not self.writer.is_closing():
                self.writer.write(data)
                self.last_write = time.monotonic()

    def _release(self) -> None:
        now = time.monotonic()
        while self._delayed and self._delayed[0][0] <= now + 1e-4:
            _due, data = self._delayed.popleft()
            if not self.writer.is_closing():
                self.writer.write(data)
                self.last_write = now
        if self._delayed:
            asyncio.get_running_loop().call_later(max(0.0, self._delayed[0][0] - now), self._release)

    def send_method(self, ch: int, m: Method) -> None:
        self.send(codec.method_frame(ch, m))


class _FrameProtocol(asyncio.Protocol):
    """A broker connection after the protocol header: every read is parsed
    and handled synchronously in the transport callback.  Write flow control
    and connection loss are forwarded to the StreamWriter's protocol."""

    def __init__(self, broker: "Broker", c: _ServerConn, transport: asyncio.Transport) -> None:
        self.broker, self.c, self.tr = broker, c, transport
        self.old = transport.get_protocol()
        self.parser = codec.FrameParser()
        self.done: asyncio.Future = asyncio.get_running_loop().create_future()

    def data_received(self, data: bytes) -> None:
        if self.done.done():
            return
        self.c.last_read = time.monotonic()
        try:
            ok = self.broker._frames(self.c, self.parser.feed(data))
        except codec.FrameError:
            ok = False
        if not ok:
            self.tr.pause_reading()
            self.done.set_result(None)

    def eof_received(self) -> bool:
        if not self.done.done():
            self.done.set_result(None)
        return False

    def connection_lost(self, exc) -> None:
        if not self.done.done():
            self.done.set_result(None)
        self.old.connection_lost(exc)

    def pause_writing(self) -> None:
        self.old.pause_writing()

    def resume_writing(self) -> None:
        self.old.resume_writing()


class Broker:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, *, username: str | None = None,
                 password: str | None = None, heartbeat: int = 0, frame_max: int = codec.DEFAULT_FRAME_MAX) -> None:
        self.host = host
        self.port = port
        self.username = username
        self.password = password
        self.heartbeat = heartbeat
        self.frame_max = frame_max
        self.exchanges: dict[str, Exchange] = {"": Exchange("", "direct", True),
                                               "amq.direct": Exchange("amq.direct", "direct", True),
                                               "amq.fanout": Exchange("amq.fanout", "fanout", True),
                                               "amq.topic": Exchange("amq.topic", "topic", True)}
        self.queues: dict[str, Queue] = {}
        self.conns: set[_ServerConn] = set()
        self._server: asyncio.AbstractServer | None = None
        self._ctag = itertools.count(1)
        self._qname = itertools.count(1)
        self.blocked = False
        self.delivery_paused = False
        # RabbitMQ's consumer_timeout (3.8.15+, 30 min by default there; None = off): a
        # delivery left unacked longer closes its channel with 406 PRECONDITION_FAILED
        self.consumer_timeout: float | None = None
        self._timeout_task: asyncio.Task | None = None
        self.fail_publishes = 0
        self.confirm_delay = 0.0           # fault injection: publisher confirms arrive this much later
        self.events: list[tuple[str, str]] = []   # ("publish", exchange) / ("ack", queue), in order
        self.published: list[QMsg] = []
        self.stats = collections.Counter()
        self.users: dict[str, tuple[str, Perms]] = {}
        self.refusals: list[tuple[str, str, str, str]] = []   # (user, kind, resource type, name)
        from .rawserver import fake_rtt
        self.rtt = fake_rtt()              # emulated round trip: every frame sent arrives this much later

    def add_user(self, user: str, password: str, *, configure: str = ".*", write: str = ".*",
                 read: str = ".*") -> None:
        """A login with its own permission regexes (``rabbitmqctl set_permissions``)."""
        self.users[user] = (password, Perms(configure, write, read))

    def _check(self, c: "_ServerConn", kind: str, rtype: str, name: str, m: Method) -> None:
        if c.perms is None:
            return
        rname = "amq.default" if rtype == "exchange" and name == "" else name
        if not c.perms.allows(kind, rname):
            self.refusals.append((c.user, kind, rtype, rname))
            self.stats["refused"] += 1
            raise ChannelError(codec.ACCESS_REFUSED,
                               f"ACCESS_REFUSED - {kind} access to {rtype} '{rname}' in vhost '/' "
                               f"refused for user '{c.user}'", m.ids)

    # ------------------------------------------------------------ lifecycle
    async def start(self) -> "Broker":
        self._server = await asyncio.start_server(self._handle, self.host, self.port)
        self.port = self._server.sockets[0].getsockname()[1]
        self._timeout_task = asyncio.ensure_future(self._consumer_timeouts())
        return self

    async def _consumer_timeouts(self) -> None:
        """rabbit_channel's delivery-acknowledgement timeout: a channel holding
        a consumer delivery unacked for longer than ``consumer_timeout`` is
        closed with 406 (its unacked deliveries go back to their queues)."""
        try:
            while True:
                to = self.consumer_timeout
                await asyncio.sleep(min(0.05, to / 4) if to else 0.2)
                if not to:
                    continue
                now = time.monotonic()
                for c in list(self.conns):
                    for sc in list(c.channels.values()):
                        old = [t for t, at in sc.delivered_at.items() if now - at > to and t in sc.unacked
                               and sc.unacked[t][2] is not None]
                        if not old:
                            continue
                        self.stats["consumer_timeouts"] += 1
                        c.channels.pop(sc.id, None)
                        self._close_channel(sc)
                        c.send_method(sc.id, Method("channel.close", {
                            "reply_code": codec.PRECONDITION_FAILED,
                            "reply_text": f"PRECONDITION_FAILED - delivery acknowledgement on channel {sc.id} "
                                          f"timed out. Timeout value used: {int(to * 1000)} ms. This timeout "
                                          "value can be configured, see consumers doc guide to learn more",
                            "class_id": 0, "method_id": 0}))
        except asyncio.CancelledError:
            pass

    @property
    def url(self) -> str:
        u = self.username or "guest"
        p = self.password or "guest"
        return f"amqp://{u}:{p}@{self.host}:{self.port}/"

    @property
    def endpoint(self) -> str:
        return f"{self.host}:{self.port}"

    async def stop(self) -> None:
        if self._timeout_task is not None:
            self._timeout_task.cancel()
            self._timeout_task = None
        if self._server is not None:
            self._server.close()
            await self.drop_connections()
            await self._server.wait_closed()
            self._server = None

    async def drop_connections(self, code: int = codec.CONNECTION_FORCED, text: str = "broker forced close",
                               graceful: bool = False) -> None:
        """Fault injection: kill every client connection (unacked messages are requeued)."""
        for c in list(self.conns):
            if graceful:
                c.send_method(0, Method("connection.close", {"reply_code": code, "reply_text": text}))
            if graceful:
                c.flush()
            self._teardown(c)
            try:
                c.writer.transport.abort() if not graceful else c.writer.close()
            except Exception:
                pass
        await asyncio.sleep(0)

    def set_blocked(self, blocked: bool) -> None:
        self.blocked = blocked
        for c in self.conns:
            if c.open:
                c.send_method(0, Method("connection.blocked", {"reason": "low on memory"}) if blocked
                              else Method("connection.unblocked"))

    def delete_queue(self, name: str) -> int:
        """Delete a queue from outside any connection (an operator's
        ``rabbitmqctl delete_queue``): its consumers get ``basic.cancel``."""
        q = self.queues.pop(name, None)
        if q is None:
            return 0
        for cons in list(q.consumers):
            cons.ch.conn.send_method(cons.ch.id, Method("basic.cancel", {"consumer_tag": cons.tag}))
            self._remove_consumer(cons)
        for ex in self.exchanges.values():
            ex.bindings = [b for b in ex.bindings if b[0] != name]
        return len(q.messages)

    def delete_exchange(self, name: str) -> bool:
        """Delete an exchange from outside any connection (an operator's
        ``rabbitmqctl``/management-UI delete): publishing to it is then a
        404 channel error until someone declares it again."""
        return self.exchanges.pop(name, None) is not None

    def unbind_queue(self, name: str) -> int:
        """Remove every binding of queue ``name`` (an operator's mistake, a
        policy change): publishes routed to it are unroutable until someone
        binds it again; its messages stay.  Returns the bindings removed."""
        n = 0
        for ex in self.exchanges.values():
            keep = [b for b in ex.bindings if b[0] != name]
            n += len(ex.bindings) - len(keep)
            ex.bindings = keep
        return n

    def pause_delivery(self, paused: bool) -> None:
        """Fault injection: consumers stay registered but get nothing (a stuck
        queue process); resuming dispatches what queued up meanwhile."""
        self.delivery_paused = paused
        if not paused:
            for q in list(self.queues.values()):
                self._dispatch(q)

    def fail_next_publishes(self, n: int) -> None:
        """Fault injection: nack the next ``n`` confirmed publishes."""
        self.fail_publishes = n

    # ------------------------------------------------------------ introspection
    def queue_depth(self, name: str) -> int:
        q = self.queues.get(name)
        return len(q.messages) if q else 0

    def unacked_count(self) -> int:
        return sum(len(ch.unacked) for c in self.conns for ch in c.channels.values())

    def drain_queue(self, name: str) -> list[QMsg]:
        q = self.queues.get(name)
        if q is None:
            return []
        out = list(q.messages)
        q.messages.clear()
        return out

    def declare(self, topic: str, shards: int = 2, *, queue_args: dict | None = None) -> None:
        """Pre-declare a durable direct exchange ``topic`` with shard queues
        ``topic-0..`` bound by name, as another service (e.g. the converter)
        would — with its own queue arguments (``{"x-queue-type": "quorum"}``)."""
        ex = self.exchanges.setdefault(topic, Exchange(topic, "direct", True))
        for i in range(shards):
            q = f"{topic}-{i}"
            self.queues.setdefault(q, Queue(q, True, arguments=dict(queue_args or {})))
            if (q, q, {}) not in ex.bindings:
                ex.bindings.append((q, q, {}))

    def inject(self, exchange: str, routing_key: str, body: bytes, props: Properties | None = None) -> int:
        """Publish from outside any connection (test producer). Returns #queues routed."""
        return self._route(QMsg(body, props or Properties(), exchange, routing_key))

    # ------------------------------------------------------------ connection
    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        c = _ServerConn(self, reader, writer)
        self.conns.add(c)
        try:
            hdr = await reader.readexactly(8)
            if self.rtt:
                await asyncio.sleep(self.rtt)      # the TCP handshake before the protocol header
            if hdr != codec.PROTOCOL_HEADER:
                writer.write(codec.PROTOCOL_HEADER)
                return
            c.send_method(0, Method("connection.start", {
                "version_major": 0, "version_minor": 9,
                "server_properties": {"product": "tritondl-fakebroker", "version": "3.8-compat",
                                      "capabilities": {"publisher_confirms": True, "basic.nack": True,
                                                       "consumer_cancel_notify": True,
                                                       "connection.blocked": True, "per_consumer_qos": True}},
                "mechanisms": b"PLAIN AMQPLAIN", "locales": b"en_US"}))
            # from here on frames are handled inside the transport's read callback
            # (no StreamReader buffer, no task wake-up per read): the broker's cost
            # per message is what bounds a node of competing workers
            proto = _FrameProtocol(self, c, writer.transport)
            leftover = bytes(getattr(reader, "_buffer", b""))
            if hasattr(reader, "_buffer"):
                reader._buffer.clear()
            writer.transport.set_protocol(proto)
            if not writer.transport.is_reading():
                writer.transport.resume_reading()
            if leftover:
                proto.data_received(leftover)
            await proto.done
        except (asyncio.IncompleteReadError, ConnectionError, OSError, codec.FrameError):
            pass
        finally:
            self._teardown(c)
            try:
                c.flush()
                writer.close()
            except Exception:
                pass

    def _frames(self, c: _ServerConn, frames) -> bool:
        """Handle parsed frames; False once the connection is to be closed."""
        for ftype, ch, payload in frames:
            try:
                self._on_frame(c, ftype, ch, payload)
            except ConnError as e:
                c.send_method(0, Method("connection.close", {"reply_code": e.code,
                                                             "reply_text": e.text[:255],
                                                             "class_id": e.cm[0], "method_id": e.cm[1]}))
                c.flush()
                return False
            except ChannelError as e:
                sc = c.channels.pop(ch, None)
                if sc is not None:
                    self._close_channel(sc)
                c.send_method(ch, Method("channel.close", {"reply_code": e.code, "reply_text": e.text[:255],
                                                           "class_id": e.cm[0], "method_id": e.cm[1]}))
            if c.closed:
                return False
        return True

    async def _heartbeats(self, c: _ServerConn) -> None:
        """RabbitMQ's side of heartbeats: a frame every hb/2 s of write
        silence, and a connection with 2*hb s of read silence is dead."""
        hb = c.hb
        try:
            while not c.closed:
                await asyncio.sleep(hb / 2)
                now = time.monotonic()
                if now - c.last_write >= hb / 2:
                    c.send(codec.HEARTBEAT_FRAME)
                    self.stats["heartbeats_sent"] += 1
                if now - c.last_read > 2 * hb:
                    self.stats["heartbeat_timeouts"] += 1
                    self._teardown(c)
                    try:
                        c.writer.transport.abort()
                    except Exception:
                        pass
                    return
        except asyncio.CancelledError:
            pass

    def _teardown(self, c: _ServerConn) -> None:
        if c in self.conns:
            self.conns.discard(c)
        c.closed = True
        if c.hb_task is not None and c.hb_task is not asyncio.current_task():
            c.hb_task.cancel()
        for ch in list(c.channels.values()):
            self._close_channel(ch)
        c.channels.clear()
        for q in [q for q in self.queues.values() if q.exclusive and q.owner is c]:
            self.queues.pop(q.name, None)

    def _close_channel(self, ch: _ServerChannel) -> None:
        for cons in list(ch.consumers.values()):
            self._remove_consumer(cons)
        # requeue unacked in original order, marked redelivered
        for tag in sorted(ch.unacked, reverse=True):
            msg, q, _cons = ch.unacked[tag]
            msg.redelivered = True
            if q.name in self.queues:
                q.messages.appendleft(msg)
        touched = {q.name for _m, q, _c in ch.unacked.values()}
        ch.unacked.clear()
        ch.delivered_at.clear()
        for name in touched:
            if name in self.queues:
                self._dispatch(self.queues[name])

    def _remove_consumer(self, cons: _Consumer) -> None:
        cons.queue.last_used = time.monotonic()
        if cons in cons.queue.consumers:
            cons.queue.consumers.remove(cons)
        cons.ch.consumers.pop(cons.tag, None)
        if cons.queue.auto_delete and not cons.queue.consumers and cons.queue.name in self.queues:
            self.queues.pop(cons.queue.name, None)

    # ------------------------------------------------------------ frames
    def _on_frame(self, c: _ServerConn, ftype: int, ch: int, payload: bytes) -> None:
        if ftype == codec.FRAME_HEARTBEAT:
            return
        if ftype == codec.FRAME_METHOD:
            m = codec.decode_method(payload)
            if ch == 0:
                self._on_conn_method(c, m)
                return
            if m.name == "channel.open":
                if ch in c.channels:
                    raise ConnError(codec.CHANNEL_ERROR, "channel already open", m.ids)
                c.channels[ch] = _ServerChannel(c, ch)
                c.send_method(ch, Method("channel.open_ok", {"channel_id": b""}))
                return
            sc = c.channels.get(ch)
            if sc is None:
                if m.name == "channel.close_ok":
                    return
                raise ConnError(codec.CHANNEL_ERROR, f"channel {ch} not open", m.ids)
            if m.name in codec.CONTENT_METHODS:
                sc.pending = (m, None, 0, [])
                return
            self._on_chan_method(c, sc, m)
        elif ftype == codec.FRAME_HEADER:
            sc = c.channels.get(ch)
            if sc is None or sc.pending is None:
                raise ConnError(codec.UNEXPECTED_FRAME, "unexpected header frame")
            _cid, size, props = codec.decode_header(payload)
            sc.pending = (sc.pending[0], props, size, [])
            if size == 0:
                self._publish(c, sc)
        elif ftype == codec.FRAME_BODY:
            sc = c.channels.get(ch)
            if sc is None or sc.pending is None or sc.pending[1] is None:
                raise ConnError(codec.UNEXPECTED_FRAME, "unexpected body frame")
            sc.pending[3].append(payload)
            if sum(len(p) for p in sc.pending[3]) >= sc.pending[2]:
                self._publish(c, sc)

    def _on_conn_method(self, c: _ServerConn, m: Method) -> None:
        n = m.name
        if n == "connection.start_ok":
            c.client_properties = m.client_properties
            resp = m.response
            if m.mechanism == "PLAIN":
                parts = resp.split(b"\x00")
                user, pw = (parts[1].decode(), parts[2].decode()) if len(parts) == 3 else ("", "")
            else:  # AMQPLAIN: a field table without its length prefix
                t = codec._Reader(struct_pack_len(resp)).table()
                user, pw = str(t.get("LOGIN", "")), str(t.get("PASSWORD", ""))
            if user in self.users:
                if pw != self.users[user][0]:
                    raise ConnError(codec.ACCESS_REFUSED, "ACCESS_REFUSED - Login was refused", m.ids)
                c.perms = self.users[user][1]
            elif (self.username is not None and (user != self.username or pw != (self.password or ""))) or \
                    (self.users and self.username is None):
                raise ConnError(codec.ACCESS_REFUSED, "ACCESS_REFUSED - Login was refused", m.ids)
            c.user = user
            c.send_method(0, Method("connection.tune", {"channel_max": 2047, "frame_max": self.frame_max,
                                                        "heartbeat": self.heartbeat}))
        elif n == "connection.tune_ok":
            c.frame_max = m.frame_max or self.frame_max
            c.hb = m.heartbeat or 0
        elif n == "connection.open":
            c.open = True
            c.send_method(0, Method("connection.open_ok"))
            if c.hb > 0:
                c.hb_task = asyncio.ensure_future(self._heartbeats(c))
            if self.blocked:
                c.send_method(0, Method("connection.blocked", {"reason": "low on memory"}))
        elif n == "connection.close":
            c.send_method(0, Method("connection.close_ok"))
            c.closed = True
        elif n == "connection.close_ok":
            c.closed = True

    def _on_chan_method(self, c: _ServerConn, ch: _ServerChannel, m: Method) -> None:
        n = m.name
        a = m.args
        ok = lambda name, **kw: c.send_method(ch.id, Method(name, kw))  # noqa: E731
        if n == "channel.close":
            c.channels.pop(ch.id, None)
            self._close_channel(ch)
            ok("channel.close_ok")
        elif n == "channel.flow":
            ch.flow = a["active"]
            ok("channel.flow_ok", active=ch.flow)
            for cons in ch.consumers.values():
                self._dispatch(cons.queue)
        elif n == "basic.qos":
            if a["global_"]:
                ch.prefetch_channel = a["prefetch_count"]
            else:
                ch.prefetch_consumer = a["prefetch_count"]
            ok("basic.qos_ok")
        elif n == "exchange.declare":
            if not a["passive"]:
                self._check(c, "configure", "exchange", a["exchange"], m)
            self._exchange_declare(m)
            if not a["nowait"]:
                ok("exchange.declare_ok")
        elif n == "exchange.delete":
            self._check(c, "configure", "exchange", a["exchange"], m)
            if a["exchange"] not in self.exchanges:
                raise ChannelError(codec.NOT_FOUND, f"NOT_FOUND - no exchange '{a['exchange']}'", m.ids)
            self.exchanges.pop(a["exchange"])
            if not a["nowait"]:
                ok("exchange.delete_ok")
        elif n == "queue.declare":
            if not a["passive"]:
                self._check(c, "configure", "queue", a["queue"], m)
                dlx = (a["arguments"] or {}).get("x-dead-letter-exchange")
                if isinstance(dlx, str):
                    self._check(c, "read", "queue", a["queue"], m)
                    self._check(c, "write", "exchange", dlx, m)
            q = self._queue_declare(c, m)
            if not a["nowait"]:
                ok("queue.declare_ok", queue=q.name, message_count=len(q.messages), consumer_count=len(q.consumers))
        elif n == "queue.bind":
            self._check(c, "write", "queue", a["queue"], m)
            self._check(c, "read", "exchange", a["exchange"], m)
            q = self._get_queue(a["queue"], m)
            ex = self.exchanges.get(a["exchange"])
            if ex is None:
                raise ChannelError(codec.NOT_FOUND, f"NOT_FOUND - no exchange '{a['exchange']}'", m.ids)
            b = (q.name, a["routing_key"], a["arguments"] or {})
            if b not in ex.bindings:
                ex.bindings.append(b)
            if not a["nowait"]:
                ok("queue.bind_ok")
        elif n == "queue.unbind":
            self._check(c, "write", "queue", a["queue"], m)
            self._check(c, "read", "exchange", a["exchange"], m)
            ex = self.exchanges.get(a["exchange"])
            if ex is not None:
                ex.bindings = [b for b in ex.bindings if not (b[0] == a["queue"] and b[1] == a["routing_key"])]
            ok("queue.unbind_ok")
        elif n == "queue.purge":
            self._check(c, "read", "queue", a["queue"], m)
            q = self._get_queue(a["queue"], m)
            cnt = len(q.messages)
            q.messages.clear()
            if not a["nowait"]:
                ok("queue.purge_ok", message_count=cnt)
        elif n == "queue.delete":
            self._check(c, "configure", "queue", a["queue"], m)
            q = self.queues.get(a["queue"])
            if q is None:
                # RabbitMQ: deleting a queue that does not exist succeeds (rabbit_channel
                # answers delete_ok with message_count 0)
                if not a["nowait"]:
                    ok("queue.delete_ok", message_count=0)
                return
            cnt = len(q.messages)
            for cons in list(q.consumers):
                cons.ch.conn.send_method(cons.ch.id, Method("basic.cancel", {"consumer_tag": cons.tag}))
                self._remove_consumer(cons)
            self.queues.pop(q.name, None)
            for ex in self.exchanges.values():
                ex.bindings = [b for b in ex.bindings if b[0] != q.name]
            if not a["nowait"]:
                ok("queue.delete_ok", message_count=cnt)
        elif n == "basic.consume":
            self._check(c, "read", "queue", a["queue"], m)
            q = self._get_queue(a["queue"], m)
            qtype = q.arguments.get("x-queue-type")
            if qtype in ("quorum", "stream") and ch.prefetch_channel > 0:
                # rabbit_channel: {error, global_qos_not_supported_for_queue_type} ->
                # protocol_error(not_implemented, ...); 540 is a hard (connection) error
                self.stats["refused_global_qos"] += 1
                raise ConnError(codec.NOT_IMPLEMENTED,
                                f"NOT_IMPLEMENTED - queue '{q.name}' in vhost '/' does not support global qos", m.ids)
            if qtype == "stream" and not ch.prefetch_consumer:
                raise ChannelError(codec.PRECONDITION_FAILED,
                                   f"PRECONDITION_FAILED - consumer prefetch count is not set for '{q.name}'", m.ids)
            if a["exclusive"] and q.consumers:
                raise ChannelError(codec.ACCESS_REFUSED, "ACCESS_REFUSED - queue in use", m.ids)
            tag = a["consumer_tag"] or f"amq.ctag-{next(self._ctag)}"
            if tag in ch.consumers:
                raise ConnError(codec.NOT_ALLOWED, "NOT_ALLOWED - attempt to reuse consumer tag", m.ids)
            cons = _Consumer(ch, tag, q, a["no_ack"], ch.prefetch_consumer)
            ch.consumers[tag] = cons
            q.consumers.append(cons)
            if not a["nowait"]:
                ok("basic.consume_ok", consumer_tag=tag)
            self._dispatch(q)
        elif n == "basic.cancel":
            cons = ch.consumers.get(a["consumer_tag"])
            if cons is not None:
                self._remove_consumer(cons)
            if not a["nowait"]:
                ok("basic.cancel_ok", consumer_tag=a["consumer_tag"])
        elif n in ("basic.ack", "basic.nack", "basic.reject"):
            self._settle(ch, m)
        elif n == "basic.get":
            self._check(c, "read", "queue", a["queue"], m)
            q = self._get_queue(a["queue"], m)
            q.last_used = time.monotonic()
            if not q.messages:
                ok("basic.get_empty")
            else:
                msg = q.messages.popleft()
                tag = next(ch.tags)
                if not a["no_ack"]:
                    ch.unacked[tag] = (msg, q, None)
                c.send(b"".join(codec.content_frames(ch.id, Method("basic.get_ok", {
                    "delivery_tag": tag, "redelivered": msg.redelivered, "exchange": msg.exchange,
                    "routing_key": msg.routing_key, "message_count": len(q.messages)}), msg.body, msg.props,
                    c.frame_max)))
        elif n in ("basic.recover", "basic.recover_async"):
            self._close_channel_unacked_only(ch)
            if n == "basic.recover":
                ok("basic.recover_ok")
        elif n == "confirm.select":
            ch.confirm = True
            if not a["nowait"]:
                ok("confirm.select_ok")
        else:
            raise ConnError(codec.NOT_IMPLEMENTED, f"method {n} not implemented", m.ids)

    def _close_channel_unacked_only(self, ch: _ServerChannel) -> None:
        for tag in sorted(ch.unacked, reverse=True):
            msg, q, cons = ch.unacked.pop(tag)
            ch.delivered_at.pop(tag, None)
            if cons:
                cons.unacked -= 1
            msg.redelivered = True
            q.messages.appendleft(msg)
            self._dispatch(q)

    # ------------------------------------------------------------ entities
    def _exchange_declare(self, m: Method) -> None:
        a = m.args
        name = a["exchange"]
        ex = self.exchanges.get(name)
        if a["passive"]:
            if ex is None:
                raise ChannelError(codec.NOT_FOUND, f"NOT_FOUND - no exchange '{name}'", m.ids)
            return
        if name.startswith("amq.") and ex is None:
            raise ChannelError(codec.ACCESS_REFUSED, "ACCESS_REFUSED - reserved name", m.ids)
        if a["type"] not in ("direct", "fanout", "topic", "headers"):
            raise ConnError(codec.COMMAND_INVALID, f"COMMAND_INVALID - unknown exchange type '{a['type']}'", m.ids)
        if ex is not None:
            if ex.type != a["type"] or ex.durable != a["durable"] or ex.auto_delete != a["auto_delete"] or \
                    ex.internal != a["internal"]:
                raise ChannelError(codec.PRECONDITION_FAILED,
                                   f"PRECONDITION_FAILED - inequivalent arg for exchange '{name}'", m.ids)
            return
        self.exchanges[name] = Exchange(name, a["type"], a["durable"], a["auto_delete"], a["internal"],
                                        a["arguments"] or {})

    def _queue_declare(self, c: _ServerConn, m: Method) -> Queue:
        a = m.args
        name = a["queue"] or f"amq.gen-{next(self._qname)}"
        q = self.queues.get(name)
        if a["passive"]:
            if q is None:
                raise ChannelError(codec.NOT_FOUND, f"NOT_FOUND - no queue '{name}'", m.ids)
            return q
        if q is not None:
            if q.exclusive and q.owner is not c:
                raise ChannelError(codec.RESOURCE_LOCKED, "RESOURCE_LOCKED - exclusive queue", m.ids)
            if q.durable != a["durable"] or q.auto_delete != a["auto_delete"] or \
                    (q.arguments or {}) != (a["arguments"] or {}):
                raise ChannelError(codec.PRECONDITION_FAILED,
                                   f"PRECONDITION_FAILED - inequivalent arg for queue '{name}'", m.ids)
            q.last_used = time.monotonic()
            return q
        q = Queue(name, a["durable"], a["exclusive"], a["auto_delete"], a["arguments"] or {},
                  owner=c if a["exclusive"] else None)
        self.queues[name] = q
        exp = q.arguments.get("x-expires")
        if isinstance(exp, int) and not isinstance(exp, bool) and exp > 0:
            self._schedule_queue_expiry(q, exp / 1000.0)
        return q

    def _schedule_queue_expiry(self, q: Queue, after: float) -> None:
        try:
            asyncio.get_running_loop().call_later(after, self._expire_queue, q)
        except RuntimeError:
            pass

    def _expire_queue(self, q: Queue) -> None:
        """RabbitMQ's ``x-expires``: a queue with no consumers that nobody has
        declared or polled for that long is deleted, and its messages are
        discarded (not dead-lettered)."""
        if self.queues.get(q.name) is not q:
            return
        ttl = q.arguments["x-expires"] / 1000.0
        idle = time.monotonic() - q.last_used
        if q.consumers or idle < ttl:
            self._schedule_queue_expiry(q, ttl if q.consumers else ttl - idle)
            return
        self.queues.pop(q.name, None)
        for ex in self.exchanges.values():
            ex.bindings = [b for b in ex.bindings if b[0] != q.name]
        self.stats["queues_expired"] += 1
        self.stats["expired_discarded"] += len(q.messages)

    def _get_queue(self, name: str, m: Method) -> Queue:
        q = self.queues.get(name)
        if q is None:
            raise ChannelError(codec.NOT_FOUND, f"NOT_FOUND - no queue '{name}'", m.ids)
        return q

    # ------------------------------------------------------------ messages
    def _route(self, msg: QMsg) -> int:
        ex = self.exchanges.get(msg.exchange)
        if ex is None:
            return -1
        targets: list[str] = []
        if msg.exchange == "":
            if msg.routing_key in self.queues:
                targets = [msg.routing_key]
        else:
            for qname, rk, _args in ex.bindings:
                if ex.type == "fanout" or (ex.type == "direct" and rk == msg.routing_key) or \
                        (ex.type == "topic" and _topic_match(rk, msg.routing_key)):
                    if qname not in targets:
                        targets.append(qname)
        for t in targets:
            q = self.queues.get(t)
            if q is None:
                continue
            qm = QMsg(msg.body, msg.props, msg.exchange, msg.routing_key)
            ttl = self._ttl_ms(q, msg.props)
            if ttl is not None:
                qm.expires_at = time.monotonic() + ttl / 1000.0
                self._schedule_expiry(q.name, ttl / 1000.0)
            q.messages.append(qm)
            self._dispatch(q)
        self.stats["routed"] += len(targets)
        return len(targets)

    def _publish(self, c: _ServerConn, ch: _ServerChannel) -> None:
        assert ch.pending is not None
        m, props, _size, parts = ch.pending
        ch.pending = None
        msg = QMsg(b"".join(parts), props or Properties(), m.exchange, m.routing_key)
        self.stats["published"] += 1
        if ch.confirm:
            ch.pub_seq += 1
        self._check(c, "write", "exchange", m.exchange, m)   # before the lookup, as rabbit_channel
        if m.exchange not in self.exchanges:
            raise ChannelError(codec.NOT_FOUND, f"NOT_FOUND - no exchange '{m.exchange}'", (60, 40))
        if ch.confirm and self.fail_publishes > 0:
            self.fail_publishes -= 1
            c.send_method(ch.id, Method("basic.nack", {"delivery_tag": ch.pub_seq}))
            return
        self.published.append(msg)
        self.events.append(("publish", m.exchange))
        n = self._route(msg)
        if n == 0 and m.mandatory:
            c.send(b"".join(codec.content_frames(ch.id, Method("basic.return", {
                "reply_code": codec.NO_ROUTE, "reply_text": "NO_ROUTE", "exchange": m.exchange,
                "routing_key": m.routing_key}), msg.body, msg.props, c.frame_max)))
        if ch.confirm:
            if self.confirm_delay:
                def confirm(tag=ch.pub_seq, ex=m.exchange) -> None:
                    self.events.append(("confirm", ex))
                    c.send_method(ch.id, Method("basic.ack", {"delivery_tag": tag}))
                asyncio.get_running_loop().call_later(self.confirm_delay, confirm)
            else:
                c.send_method(ch.id, Method("basic.ack", {"delivery_tag": ch.pub_seq}))

    def _can_deliver(self, cons: _Consumer) -> bool:
        ch = cons.ch
        if ch.conn.closed or not ch.flow:
            return False
        if cons.no_ack:
            return True
        if ch.prefetch_channel and ch.channel_unacked() >= ch.prefetch_channel:
            return False
        if cons.prefetch and cons.unacked >= cons.prefetch:
            return False
        return True

    @staticmethod
    def _ttl_ms(q: Queue, props: Properties) -> int | None:
        """Effective TTL: the lower of queue ``x-message-ttl`` and the message's
        ``expiration`` (a decimal string of milliseconds, RabbitMQ's reading)."""
        ttls = []
        qt = q.arguments.get("x-message-ttl")
        if isinstance(qt, int) and not isinstance(qt, bool) and qt >= 0:
            ttls.append(qt)
        exp = getattr(props, "expiration", None)
        if exp:
            try:
                ttls.append(max(0, int(exp)))
            except ValueError:
                pass
        return min(ttls) if ttls else None

    def _schedule_expiry(self, qname: str, delay: float) -> None:
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:
            return
        loop.call_later(delay + 0.001, self._expire_head, qname)

    def _expire_head(self, qname: str) -> None:
        """Expire messages at the queue head (RabbitMQ only expires there) and
        dead-letter them with reason ``expired``."""
        q = self.queues.get(qname)
        if q is None:
            return
        now = time.monotonic()
        while q.messages and q.messages[0].expires_at is not None and q.messages[0].expires_at <= now:
            msg = q.messages.popleft()
            self.stats["expired"] += 1
            self._dead_letter(q, msg, "expired")
        if q.messages and q.messages[0].expires_at is not None:
            self._schedule_expiry(qname, max(0.0, q.messages[0].expires_at - now))

    def _dispatch(self, q: Queue) -> None:
        if self.delivery_paused:
            return
        if q.messages and q.messages[0].expires_at is not None and q.messages[0].expires_at <= time.monotonic():
            self._expire_head(q.name)
        while q.messages and q.consumers:
            n = len(q.consumers)
            chosen = None
            for i in range(n):
                cons = q.consumers[(q.rr + i) % n]
                if self._can_deliver(cons):
                    chosen = cons
                    q.rr = (q.rr + i + 1) % n
                    break
            if chosen is None:
                return
            msg = q.messages.popleft()
            ch = chosen.ch
            tag = next(ch.tags)
            if not chosen.no_ack:
                ch.unacked[tag] = (msg, q, chosen)
                ch.delivered_at[tag] = time.monotonic()
                chosen.unacked += 1
            q.delivered_total += 1
            ch.conn.send(b"".join(codec.content_frames(ch.id, Method("basic.deliver", {
                "consumer_tag": chosen.tag, "delivery_tag": tag, "redelivered": msg.redelivered,
                "exchange": msg.exchange, "routing_key": msg.routing_key}), msg.body, msg.props,
                ch.conn.frame_max)))

    def _settle(self, ch: _ServerChannel, m: Method) -> None:
        tag = m.delivery_tag
        multiple = m.args.get("multiple", False)
        requeue = m.args.get("requeue", m.name != "basic.ack")
        if m.name == "basic.ack":
            requeue = False
        if multiple:
            tags = sorted(t for t in ch.unacked if t <= tag) if tag else sorted(ch.unacked)
        else:
            if tag not in ch.unacked:
                raise ChannelError(codec.PRECONDITION_FAILED, f"PRECONDITION_FAILED - unknown delivery tag {tag}",
                                   m.ids)
            tags = [tag]
        touched: set[str] = set()
        for t in tags:
            msg, q, cons = ch.unacked.pop(t)
            ch.delivered_at.pop(t, None)
            if cons is not None:
                cons.unacked -= 1
            touched.add(q.name)
            if m.name == "basic.ack":
                self.stats["acked"] += 1
                self.events.append(("ack", q.name))
                continue
            if requeue:
                msg.redelivered = True
                q.messages.appendleft(msg)
                self.stats["requeued"] += 1
            else:
                self.stats["dead"] += 1
                self._dead_letter(q, msg)
        for name in touched:
            if name in self.queues:
                self._dispatch(self.queues[name])
        for cons in ch.consumers.values():
            self._dispatch(cons.queue)

    def _dead_letter(self, q: Queue, msg: QMsg, reason: str = "rejected") -> None:
        dlx = q.arguments.get("x-dead-letter-exchange")
        if dlx is None:
            self.stats["dropped"] += 1
            return
        rk = q.arguments.get("x-dead-letter-routing-key", msg.routing_key)
        props = msg.props
        hdrs = dict(props.headers or {})
        deaths = [d for d in (hdrs.get("x-death") or []) if isinstance(d, dict)]
        prev = next((d for d in deaths if d.get("queue") == q.name and d.get("reason") == reason), None)
        if prev is not None:
            deaths.remove(prev)
        deaths.insert(0, {"queue": q.name, "reason": reason, "exchange": msg.exchange,
                          "routing-keys": [msg.routing_key], "count": (prev or {}).get("count", 0) + 1})
        hdrs["x-death"] = deaths
        # RabbitMQ strips the per-message TTL when dead-lettering (no instant re-expiry)
        new_props = Properties(**{**props.__dict__, "headers": hdrs, "expiration": None})
        self._route(QMsg(msg.body, new_props, dlx, rk))


def struct_pack_len(b: bytes) -> bytes:
    import struct
    return struct.pack(">I", len(b)) + b


async def run_broker(host: str = "127.0.0.1", port: int = 5672) -> None:  # pragma: no cover - manual use
    b = await Broker(host, port).start()
    print(f"fake broker listening on {b.endpoint}", flush=True)
    await asyncio.Event().wait()
