"""RabbitMQ job client: topology, consumer fan-in, publisher, reconnect.

Capabilities of the reference's ``internal/rabbitmq`` (components C2, C3,
C3a, C4):

* ``consume(topic)`` declares a durable **direct** exchange ``topic`` and
  ``num_shard_queues`` durable queues ``topic-0..N-1`` each bound with
  routing key == queue name (``client.go:326-357,376-378,405-422``), then
  fans every shard's deliveries into ONE stream (``client.go:242-283``).
* ``publish(topic, body)`` publishes a persistent
  ``application/octet-stream`` message round-robin over the shard routing
  keys (``client.go:189-240,386-397``).
* ``Delivery`` parses ``X-Retries`` (int32, default 0) and offers ``ack``,
  ``nack`` (no requeue) and ``retry`` (the reference's ``Error()``: ack +
  republish with ``X-Retries+1``; ``delivery.go:12-84``).
* connection loss is detected by callback + heartbeats (not 1 s polling) and
  repaired with the cenkalti exponential policy (``client.go:139-184,303-322``);
  consumers and the publisher come back on the new connection.

Fixes vs the reference: one TCP connection with one
channel per shard consumer + one confirm-mode publisher channel (B6); the
publish retry is a real capped exponential instead of ``Backoff ^ 2`` with a
self-deadlocking re-enqueue (B5); the publish exchange is declared before
first use (B13); all state lives on one event loop (B7).

QoS is per consumer (``basic.qos(prefetch, global=false)``), not the
reference's channel-wide ``Qos(prefetch, 0, true)`` (``client.go:366-369``).
Each shard has its own channel with exactly one consumer on it, so the limit
is the same number of unacked deliveries; but RabbitMQ refuses a consumer
on a quorum (or stream) queue from a channel with global QoS (540
NOT_IMPLEMENTED, which closes the connection), so per-consumer QoS is what
lets the worker consume shard queues an operator declared as quorum queues.

Every shard's consumer state is tracked (:class:`Shard`): whether it has a
live consumer and since when, and since when the connection has been lost.
``/healthz`` reads that (:meth:`Client.health`) — the reference's 1 s
scheduler re-created a dead processor (``client.go:139-166``); here the
re-creation is event-driven and the probe sees a shard that stays down.

Topology this worker does not own never blocks it.  The reference declared
nothing on the publish side (``client.go:224`` publishes straight to the
exchange), so it needed only *write* permission on ``v1.convert`` and worked
whatever arguments the converter gave its queues.  Every declare made here
beyond the reference's consume-side ones (``client.go:326-357``) is
best-effort: a 403 ACCESS_REFUSED or 406 PRECONDITION_FAILED marks the
entity as externally managed (on a scratch channel, so the confirm channel
and its in-flight publishes are untouched) and the worker goes on without
declaring it.  A retry whose delay queue cannot be declared falls back to
the reference's own ``Error()`` (``delivery.go:66-84``): wait in-process,
re-publish to the original exchange/routing key with ``X-Retries+1``, ack —
needing only the write permission the consume side already has.
"""

from __future__ import annotations

import asyncio
import contextlib
import dataclasses
import itertools
import os
import secrets
import socket
import time
from dataclasses import dataclass
from typing import AsyncIterator

from ..utils.backoff import BackoffExhausted, ExponentialBackoff
from ..utils.gocompat import durafmt
from ..utils.log import log
from . import codec
from .codec import AMQPError, Properties
from .connection import Channel, ChannelClosed, Connection, ConnectionClosed, Message, PublishReturned

ErrorEnsureExchange = "failed to ensure exchange"
ErrorEnsureConsumerQueues = "failed to ensure consumer queues"


class ConsumeError(AMQPError):
    pass


class DelayUnavailable(AMQPError):
    """The broker refused the retry delay queue (its declare or the publish into it)."""


class LeaseRefused(AMQPError):
    """The broker refused a job lease queue (no *configure* on it, or no
    *write* on the default exchange)."""


_HOLDER = f"{socket.gethostname()}:{os.getpid()}"


# channel errors that say "this topology is not yours": the entity exists with other
# arguments (406) or this user may not configure / write it (403)
_NOT_OURS = (codec.ACCESS_REFUSED, codec.PRECONDITION_FAILED)


def _refused(e: BaseException) -> bool:
    return isinstance(e, ChannelClosed) and e.code in _NOT_OURS


@dataclass
class DeliveryMetadata:
    retries: int = 0


# Headers this worker adds (the reference's own is X-Retries, delivery.go:32-44).
LEASE_RETURNS = "X-Lease-Returns"   # times the job came back because its holder's lease ran out
LEASE_HOLDER = "X-Lease-Holder"     # host:pid that holds the lease copy (diagnostics)
BUSY = "X-Busy"                     # hand-backs because another worker was running the same job
# a buffered delivery the broker had flagged redelivered, handed back by pause(): the copy is a
# fresh message, so this keeps it checked against the done-ledger like the redelivery it was
REDELIVERED = "X-Tdl-Redelivered"
OPS_CHANNELS = 8                    # idle lease-ops channels kept open


def _int_header(headers: dict | None, name: str) -> int:
    v = (headers or {}).get(name)
    return v if isinstance(v, int) and not isinstance(v, bool) and v > 0 else 0


def _lease_expired(headers: dict | None) -> bool:
    """Did this message just come back from a lease queue whose TTL ran out?
    RabbitMQ prepends the newest death to ``x-death``."""
    deaths = (headers or {}).get("x-death")
    if not isinstance(deaths, list) or not deaths or not isinstance(deaths[0], dict):
        return False
    d = deaths[0]
    return d.get("reason") == "expired" and ".lease." in str(d.get("queue", ""))


class Lease:
    """Where a leased delivery lives while its job runs: a copy in a per-job
    queue ``<rk>.lease.<token>.<n>`` whose ``x-message-ttl`` is the lease and
    whose dead-letter target is the job's own exchange and routing key."""

    def __init__(self, token: str, ttl: float) -> None:
        self.token = token
        self.ttl = ttl
        self.n = 0
        self.queue = ""
        self.lost = False                 # the copy ran out before a renewal: the job went back
        self.renewed_at = time.monotonic()


class Delivery:
    """One job message (reference ``Delivery``, ``delivery.go:17-28``).

    A delivery can be *leased* (:meth:`hold`): after ``after`` seconds the
    broker keeps a copy in a lease queue (:class:`Lease`) and the original
    is acked, so the delivery no longer sits unacked on its channel.
    RabbitMQ closes a channel that holds a delivery longer than its
    ``consumer_timeout`` (30 min by default) and requeues the delivery, and
    another worker then runs the job a second time.  The reference held
    every delivery unacked for its whole job (``cmd/downloader/
    downloader.go:103-155``), so its torrent jobs hit that timeout.  The
    lease is renewed every ``ttl / 2`` while the job runs.  If the worker
    dies, the copy expires and dead-letters back to the shard queue, so the
    job is run again.  ``ack`` / ``nack`` / ``retry`` of a leased delivery
    act on the copy."""

    def __init__(self, client: "Client", msg: Message, generation: int) -> None:
        self.client = client
        self.msg = msg
        self.generation = generation
        h = msg.properties.headers
        self.metadata = DeliveryMetadata(retries=_parse_retries(h))
        self.settled = False
        self.lease_return = _lease_expired(h)
        self.lease_returns = _int_header(h, LEASE_RETURNS) + (1 if self.lease_return else 0)
        self.busy = _int_header(h, BUSY)
        self.handed_back_redelivered = _int_header(h, REDELIVERED) > 0
        self.lease: Lease | None = None
        self.requeue_props: Properties | None = None   # what a requeue publishes (a park's retry headers)
        self._hold: asyncio.Task | None = None
        self._hold_timer: asyncio.TimerHandle | None = None
        self._lock: asyncio.Lock | None = None

    @property
    def body(self) -> bytes:
        return self.msg.body

    @property
    def exchange(self) -> str:
        return self.msg.exchange

    @property
    def routing_key(self) -> str:
        return self.msg.routing_key

    @property
    def redelivered(self) -> bool:
        return self.msg.redelivered

    @property
    def maybe_duplicate(self) -> bool:
        """Could this job have been run to the end already?  Redelivered
        (an ack went nowhere; also a redelivered delivery :meth:`Client.pause`
        handed back), back from an expired lease, or handed back because
        another worker was running it."""
        return self.msg.redelivered or self.handed_back_redelivered or self.lease_return or self.busy > 0

    @property
    def stale(self) -> bool:
        """True once the broker has taken the job back: the channel it arrived
        on is gone (the broker requeued it), or its lease ran out."""
        if self.lease is not None:
            return self.lease.lost
        return self.msg.channel is None or self.msg.channel.is_closed

    async def ack(self) -> bool:
        """``Ack`` (single, ``delivery.go:55-57``).  False if the ack could not
        be sent because the delivery's channel is gone (the broker requeues
        it: it will be delivered again), or because its lease had run out."""
        return await self._settle(lambda: self.msg.ack(), lambda: self.client._lease_release(self))

    async def nack(self, requeue: bool = False) -> None:
        """``Nack`` (single, no requeue by default, ``delivery.go:60-62``)."""
        await self._settle(lambda: self.msg.nack(requeue=requeue),
                           lambda: self.client._lease_release(self, requeue=requeue))

    def retry_props(self, increment: int = 1, *, busy: bool = False) -> Properties:
        """Headers for the next copy of this job: ``X-Retries + increment``;
        ``busy`` counts a hand-back in ``X-Busy`` (another worker runs the
        job); lease returns so far are carried in ``X-Lease-Returns``."""
        hdrs = dict(self.msg.properties.headers or {})
        hdrs["X-Retries"] = self.metadata.retries + increment
        hdrs.pop("x-death", None)
        hdrs.pop(LEASE_HOLDER, None)
        hdrs.pop(REDELIVERED, None)
        if busy:
            hdrs[BUSY] = self.busy + 1
        else:
            hdrs.pop(BUSY, None)
        if self.lease_returns:
            hdrs[LEASE_RETURNS] = self.lease_returns
        return Properties(headers=hdrs, delivery_mode=self.msg.properties.delivery_mode or codec.PERSISTENT,
                          content_type=self.msg.properties.content_type)

    def hold(self, after: float | None = None, ttl: float | None = None) -> None:
        """Lease this delivery ``after`` seconds from now unless it is settled
        by then, and renew the lease every ``ttl / 2`` until it is (defaults:
        the client's ``lease_after`` / ``lease_ttl``; off when either is 0 or
        the broker refused a lease queue for this routing key before)."""
        after = self.client.lease_after if after is None else after
        ttl = self.client.lease_ttl if ttl is None else ttl
        if self._hold is not None or self._hold_timer is not None or self.settled or after <= 0 or ttl <= 0 or \
                self.routing_key in self.client._lease_refused:
            return
        # a timer, not a task: most jobs settle long before it fires (no task per job)
        self._hold_timer = asyncio.get_running_loop().call_later(after, self._start_hold, ttl)

    def _start_hold(self, ttl: float) -> None:
        self._hold_timer = None
        if self.settled or self.client._closing:
            return
        holding = self.client._holding
        holding.add(self)
        self._hold = asyncio.ensure_future(self.client._hold(self, 0.0, ttl))
        self._hold.add_done_callback(lambda _t: holding.discard(self))

    def _settle_lock(self) -> asyncio.Lock:
        if self._lock is None:
            self._lock = asyncio.Lock()
        return self._lock

    async def retry(self, delay: float | None = None, *, increment: int = 1, busy: bool = False) -> str:
        """Reference ``Error()``: re-publish the same body with ``X-Retries + 1``
        after ``delay`` and ack (``delivery.go:66-84``).  Returns how: "now",
        "delay-queue" or "parked".

        The Go version slept its goroutine for the delay (``:72``), holding the
        job slot.  Here the wait happens in the broker: the copy is published
        (confirmed) to a per-shard delay queue whose ``x-message-ttl`` is the
        delay and whose dead-letter target is the original exchange/routing key,
        then the original is acked — the caller's slot is free at once, and a
        crash at any point duplicates the job instead of losing it.  When the
        broker refuses the delay queue (a user without *configure* on it, or a
        queue of that name with other arguments) the delivery is parked
        in-process instead (:meth:`Client.park`): the reference's own
        sleep-republish-ack, run as a task so the job slot is still free.
        ``increment=0`` hands a delivery back without spending a retry
        (``busy``: because another worker is running the same job)."""
        d = self.client.retry_delay if delay is None else delay
        props = self.retry_props(increment, busy=busy)
        if d > 0:
            log.info("retrying message in %s", durafmt(d))
            try:
                await self.client.publish_delayed(self.msg.exchange, self.msg.routing_key, self.msg.body, props, d)
            except DelayUnavailable as e:
                log.with_field("error", str(e)).warn("delay queue unavailable; waiting in-process")
                self.client.park(self, props, d)
                return "parked"
            await self.ack()
            return "delay-queue"
        await self.client.publish_raw(self.msg.exchange, self.msg.routing_key, self.msg.body, props)
        await self.ack()
        return "now"

    async def _settle(self, fn, leased_fn) -> bool:
        # under the lease lock: a lease being taken or renewed finishes first, so the
        # settlement acts on whichever of the original and the copy is the live one
        async with self._settle_lock():
            if self.settled:
                return False
            if self._hold_timer is not None:
                self._hold_timer.cancel()
                self._hold_timer = None
            if self._hold is not None:
                self._hold.cancel()      # between renewals (the lock is ours): nothing half-done
            if self.lease is not None:
                self.settled = True
                self.client._leased.discard(self)
                return await leased_fn()
            if self.stale:
                self.settled = True
                log.with_field("delivery_tag", self.msg.delivery_tag).warn(
                    "delivery's channel is gone; broker will redeliver it")
                return False
            await fn()
            self.settled = True
            self.client._unhold(self)
            return True


class Shard:
    """One shard queue's consumer: its channel and consumer tag, and since when
    it has (or has not) been consuming."""

    def __init__(self, topic: str, queue: str) -> None:
        self.topic = topic
        self.queue = queue
        self.channel: Channel | None = None
        self.tag = ""
        self.on_msg = None
        self.active = False
        self.paused = False                # consumer cancelled on purpose (Client.pause)
        self.since = time.monotonic()      # when ``active`` last changed
        self.rotations = 0                 # consumer re-subscriptions made for parked deliveries
        self.held: dict[int, str] = {}     # delivery tag -> consumer tag, delivered and not yet settled
        self.lock = asyncio.Lock()

    def set_active(self, ch: Channel, tag: str, on_msg) -> None:
        self.channel, self.tag, self.on_msg = ch, tag, on_msg
        self.paused = False
        if not self.active:
            self.active = True
            self.since = time.monotonic()

    def set_inactive(self) -> None:
        self.tag = ""
        if self.active:
            self.active = False
            self.since = time.monotonic()

    def has_room(self, prefetch: int) -> bool:
        """Could the broker deliver one more message to this shard's consumer
        (its per-consumer prefetch counts only the current consumer tag)?"""
        if not self.active:
            return False
        return prefetch <= 0 or sum(1 for t in self.held.values() if t == self.tag) < prefetch

    def down_for(self, now: float | None = None) -> float:
        """Seconds this shard has had no consumer (0 while it has one, or while
        its consumer is paused on purpose)."""
        return 0.0 if (self.active or self.paused) else (now or time.monotonic()) - self.since


def _parse_retries(headers: dict | None) -> int:
    """X-Retries must be an int32; anything else → 0 (``delivery.go:32-44``)."""
    if not headers:
        return 0
    v = headers.get("X-Retries")
    if isinstance(v, bool) or not isinstance(v, int):
        return 0
    if not -(2**31) <= v < 2**31:
        return 0
    return v


class Client:
    """``rabbitmq.NewClient`` equivalent."""

    def __init__(self, url: str, *, prefetch: int = 10, num_shard_queues: int = 2, heartbeat: int = 30,
                 backoff: ExponentialBackoff | None = None, retry_delay: float = 10.0,
                 declare_publish: bool = True, declare_publish_queues: bool = True, mandatory: bool = True) -> None:
        """``declare_publish=False`` is the reference exactly (nothing declared on
        the publish side, ``client.go:224``); with it on (default) the exchange,
        and with ``declare_publish_queues`` its shard queues, are declared
        best-effort before the first publish so messages are not lost to a
        missing exchange (B13).  ``mandatory`` (default) publishes so that a
        message no queue is bound for comes back (``basic.return``) instead of
        being confirmed and dropped; the reference's publishes were not
        mandatory (``client.go:224-240``)."""
        self.url = url
        self.prefetch = prefetch                   # reference default 10 (client.go:107)
        self.num_shard_queues = num_shard_queues   # reference: 2 (client.go:108)
        self.heartbeat = heartbeat
        self.backoff = backoff or ExponentialBackoff()
        self.retry_delay = retry_delay
        self.declare_publish = declare_publish
        self.declare_publish_queues = declare_publish_queues
        self.mandatory = mandatory
        self.returned = 0                          # publishes the broker could not route (basic.return)
        self.paused = False                        # consumers stopped by pause() (a long job holds the slots)
        self.handed_back = 0                       # buffered deliveries given back by pause()
        self.conn: Connection | None = None
        self.generation = 0
        self._topics: list[str] = []
        self._out: asyncio.Queue[Delivery | None] = asyncio.Queue()
        self._pub: Channel | None = None
        self._pub_lock = asyncio.Lock()
        self._rk_index: dict[str, itertools.cycle] = {}
        self._declared_pub: set[str] = set()
        self._declared_delay: set[str] = set()
        # entities the broker told us are not ours (403/406): never declared again
        self.external_topics: set[str] = set()
        self.external_queues: set[str] = set()
        self._refused_delay: set[str] = set()
        self._parked = 0                           # deliveries waiting in-process (park)
        self.parked_total = 0
        self.shards: dict[str, Shard] = {}         # shard queue -> its consumer state
        self.lost_since: float | None = None       # monotonic time the connection was lost (None: up)
        self.consumer_timeouts = 0                 # shard channels the broker closed for a late ack
        self.confirm_ewma: float | None = None     # publish -> broker confirm, seconds (EWMA, alpha 0.2)
        self._consumer_chans: list[Channel] = []
        # leases (Delivery.hold): taken this long after a delivery arrives, TTL of the copy
        # (renewed every ttl / 2); 0 = off, the delivery is held unacked as the reference did
        self.lease_after = 0.0
        self.lease_ttl = 0.0
        self._lease_refused: set[str] = set()      # routing keys whose lease queues the broker refused
        self._leased: set[Delivery] = set()        # leased deliveries not settled yet
        self._holding: set[Delivery] = set()       # deliveries whose lease task runs (Delivery.hold)
        self._ops_free: list[Channel] = []     # idle lease-ops channels (one RPC in flight per channel)
        self.lease_stats = {"taken": 0, "renewed": 0, "released": 0, "lost": 0, "requeued": 0, "refused": 0}
        self._closing = False
        self._bg: set[asyncio.Task] = set()
        self._connected = asyncio.Event()
        self._supervisor: asyncio.Task | None = None
        self._lost = asyncio.Event()
        self.reconnects = 0

    # ------------------------------------------------------------ connect
    def set_prefetch(self, prefetch: int) -> None:
        """``SetPrefetch`` (``client.go:381-383``); applies to channels opened afterwards."""
        self.prefetch = prefetch

    async def connect(self) -> "Client":
        await self._dial_with_backoff()
        self._supervisor = asyncio.ensure_future(self._supervise())
        return self

    async def _dial_with_backoff(self) -> None:
        pol = self.backoff
        pol.reset()
        while True:
            try:
                conn = await Connection.open(self.url, heartbeat=self.heartbeat)
                break
            except (OSError, AMQPError, asyncio.TimeoutError) as e:
                d = pol.next_delay()
                log.error("failed to dial rabbitmq: %s", e)
                if d is None or self._closing:
                    raise BackoffExhausted(f"giving up dialing rabbitmq: {e}") from e
                await asyncio.sleep(d)
        self.conn = conn
        self.generation += 1
        self._pub = None
        self._declared_pub.clear()
        self._declared_delay.clear()
        self._consumer_chans = []
        self._lost.clear()
        conn.add_close_callback(self._on_conn_lost)
        self._connected.set()

    def _on_conn_lost(self, err: BaseException) -> None:
        self._connected.clear()
        self._lost.set()
        if self.lost_since is None:
            self.lost_since = time.monotonic()
        self.paused = False                 # a reconnect consumes afresh; a pause must be taken again
        for sh in self.shards.values():
            sh.set_inactive()
            sh.paused = False
        if not self._closing:
            log.with_field("error", str(err)).warn("rabbitmq connection lost; reconnecting")

    async def _supervise(self) -> None:
        try:
            while not self._closing:
                await self._lost.wait()
                if self._closing:
                    return
                try:
                    await self._dial_with_backoff()
                except BackoffExhausted as e:
                    log.error("reconnect failed permanently: %s", e)
                    self._out.put_nowait(None)
                    return
                self.reconnects += 1
                ok = True
                for t in list(self._topics):
                    try:
                        # a broker that lost its definitions (a fresh node, non-persistent
                        # storage) gets the topology back before the consumers need it
                        await self.ensure_exchange(t)
                        await self.ensure_queues(t)
                        await self._start_consumers(t)
                    except AMQPError as e:
                        ok = False
                        log.error("failed to restart consumers for %s: %s", t, e)
                        if self.conn is not None:  # force another reconnect round
                            self.conn._abort(ConnectionClosed(0, "consumer restart failed"))
                if ok and self.connected:
                    self.lost_since = None
                log.info("reconnected to rabbitmq (generation %d)", self.generation)
        except asyncio.CancelledError:
            pass

    # ------------------------------------------------------------ topology
    def get_rk(self, topic: str, index: int) -> str:
        """``getRk``: ``fmt.Sprintf("%s-%d", topic, rkIndex)`` (``client.go:376-378``)."""
        return f"{topic}-{index}"

    async def _channel(self, qos: bool = True) -> Channel:
        await self._connected.wait()
        assert self.conn is not None
        ch = await self.conn.channel()
        if qos:
            # per-consumer limit (getChannel's Qos(prefetch, 0, true) was channel-wide; with
            # one consumer per channel the limit is the same, and quorum queues accept it)
            await ch.basic_qos(self.prefetch, 0, False)
        return ch

    async def ensure_exchange(self, topic: str) -> None:
        """``ensureExchange`` (``client.go:326-334``).  A refusal (403/406) of an
        exchange that already exists adopts it as is (passive check)."""
        ch = await self._channel(qos=False)
        try:
            await ch.exchange_declare(topic, "direct", durable=True, auto_delete=False, internal=False)
        except ChannelClosed as e:
            if not _refused(e):
                raise
            await self._adopt("exchange", topic, e)
        finally:
            if not ch.is_closed:
                await ch.close()

    async def ensure_queues(self, topic: str) -> None:
        """``ensureConsumerQueues`` (``client.go:337-357``), with the same
        adoption rule per shard queue: one declared by someone else with other
        arguments (``x-queue-type: quorum``, a DLX, ...) or one this user may
        not configure is consumed as it is, and never redeclared."""
        ch = await self._channel(qos=False)
        try:
            for i in range(self.num_shard_queues):
                q = self.get_rk(topic, i)
                if q in self.external_queues:
                    continue
                try:
                    await ch.queue_declare(q, durable=True, exclusive=False, auto_delete=False)
                    await ch.queue_bind(q, topic, q)
                except ChannelClosed as e:
                    if not _refused(e):
                        raise
                    await self._adopt("queue", q, e)
                    ch = await self._channel(qos=False)
        finally:
            if not ch.is_closed:
                await ch.close()

    async def _adopt(self, kind: str, name: str, refusal: ChannelClosed) -> None:
        """The broker refused our declare of ``name``: use it if it exists
        (passive declare needs no permission), else re-raise the refusal."""
        ch = await self._channel(qos=False)
        try:
            if kind == "exchange":
                await ch.exchange_declare(name, "direct", passive=True)
            else:
                await ch.queue_declare(name, passive=True)
        except ChannelClosed:
            raise refusal from None
        finally:
            if not ch.is_closed:
                await ch.close()
        (self.external_topics if kind == "exchange" else self.external_queues).add(name)
        log.with_fields(**{kind: name, "error": str(refusal)}).warn(
            "%s is declared by someone else; using it as it is", kind)

    # ------------------------------------------------------------ consume
    async def consume(self, topic: str) -> AsyncIterator[Delivery]:
        """Declare topology and start one consumer per shard queue; returns the fan-in stream."""
        try:
            await self.ensure_exchange(topic)
        except AMQPError as e:
            raise ConsumeError(f"{ErrorEnsureExchange}: {e}") from e
        try:
            await self.ensure_queues(topic)
        except AMQPError as e:
            raise ConsumeError(f"{ErrorEnsureConsumerQueues}: {e}") from e
        self._topics.append(topic)
        for i in range(self.num_shard_queues):
            q = self.get_rk(topic, i)
            self.shards.setdefault(q, Shard(topic, q))
        await self._start_consumers(topic)
        return self._iter()

    async def _start_consumers(self, topic: str) -> None:
        gen = self.generation
        for i in range(self.num_shard_queues):
            await self._start_shard(topic, self.get_rk(topic, i), gen)

    async def _start_shard(self, topic: str, q: str, gen: int, redeclare: bool = False) -> None:
        """One consumer channel for shard queue ``q``.  It heals itself: a
        server-side ``basic.cancel`` (queue deleted, failover) re-declares and
        re-subscribes on the same channel; an unexpected ``channel.close``
        (e.g. 406 on a late ack) reopens a channel — while the connection
        lives; connection loss is the supervisor's job."""
        ch = await self._channel(qos=True)
        if redeclare and q not in self.external_queues:
            try:
                await ch.queue_declare(q, durable=True, exclusive=False, auto_delete=False)
                await ch.queue_bind(q, topic, q)
            except ChannelClosed as e:
                if not _refused(e):
                    raise
                self._mark_external_queue(q, e)
                ch = await self._channel(qos=True)
        self._consumer_chans.append(ch)
        shard = self.shards.setdefault(q, Shard(topic, q))

        def on_msg(m: Message) -> None:
            if m.body is None:  # reference skips nil bodies (client.go:262)
                return
            shard.held[m.delivery_tag] = m.consumer_tag
            self._out.put_nowait(Delivery(self, m, gen))

        def on_cancel(tag: str) -> None:
            if shard.channel is ch and shard.tag == tag:
                shard.set_inactive()
            log.with_fields(queue=q, consumer_tag=tag).warn("consumer cancelled by broker; resubscribing")
            self._spawn_bg(self._resubscribe(topic, ch, q, on_msg, gen))

        started = False

        def on_close(exc) -> None:
            if ch in self._consumer_chans:
                self._consumer_chans.remove(ch)
            if shard.channel is ch:
                shard.set_inactive()
                shard.held.clear()          # the broker requeued them with the channel
            if getattr(exc, "code", 0) == codec.PRECONDITION_FAILED and "acknowledgement" in str(exc):
                # RabbitMQ's consumer_timeout (30 min by default): a job ran longer than the broker
                # lets a delivery sit unacked; the delivery goes back to the queue
                self.consumer_timeouts += 1
                log.with_fields(queue=q, error=str(exc)).error(
                    "the broker closed this shard's channel: a job ran longer than its consumer_timeout "
                    "allows; raise consumer_timeout (rabbitmq.conf, or the consumer-timeout policy / "
                    "x-consumer-timeout on the shard queues) above the longest job")
            if not started:
                return          # the basic.consume itself failed: the caller's retry loop owns the shard
            if self._closing or gen != self.generation or getattr(exc, "code", 0) == 200 or \
                    self.conn is None or self.conn.is_closed or isinstance(exc, ConnectionClosed):
                return
            log.with_fields(queue=q, error=str(exc)).warn("consumer channel closed by broker; reopening")
            self._spawn_bg(self._reopen_shard(topic, q, gen))

        ch.on_cancel = on_cancel
        ch.add_close_callback(on_close)
        try:
            tag = await ch.basic_consume(q, on_msg, no_ack=False)
        except BaseException:
            if not ch.is_closed:
                with contextlib.suppress(Exception):
                    await ch.close()
            raise
        started = True
        shard.set_active(ch, tag, on_msg)
        log.info("worker on queue '%s' started", q)

    def _mark_external_queue(self, q: str, e: BaseException) -> None:
        self.external_queues.add(q)
        log.with_fields(queue=q, error=str(e)).warn("queue is declared by someone else; consuming it as it is")

    def _spawn_bg(self, coro) -> None:
        t = asyncio.ensure_future(coro)
        self._bg.add(t)
        t.add_done_callback(self._bg.discard)

    async def _reopen_shard(self, topic: str, q: str, gen: int) -> None:
        pol = ExponentialBackoff(initial=0.05, max_interval=5.0, max_elapsed=None)
        while not self._closing and gen == self.generation and self.conn is not None and not self.conn.is_closed:
            try:
                await self._start_shard(topic, q, gen, redeclare=True)
                return
            except AMQPError as e:
                d = pol.next_delay() or 1.0
                log.with_fields(queue=q, error=str(e)).warn("reopening consumer failed; retrying in %.2fs", d)
                await asyncio.sleep(d)

    async def _resubscribe(self, topic: str, ch: Channel, q: str, cb, gen: int) -> None:
        pol = ExponentialBackoff(initial=0.05, max_interval=5.0, max_elapsed=None)
        while not self._closing and gen == self.generation and not ch.is_closed:
            try:
                if q not in self.external_queues:
                    try:
                        await ch.queue_declare(q, durable=True, exclusive=False, auto_delete=False)
                        await ch.queue_bind(q, topic, q)
                    except ChannelClosed as e:
                        if not _refused(e):
                            raise
                        self._mark_external_queue(q, e)
                        return          # the refusal closed ch: its close callback reopens the shard
                tag = await ch.basic_consume(q, cb, no_ack=False)
                shard = self.shards.get(q)
                if shard is not None:
                    shard.set_active(ch, tag, cb)
                log.info("worker on queue '%s' resubscribed", q)
                return
            except AMQPError as e:
                d = pol.next_delay() or 1.0
                log.with_fields(queue=q, error=str(e)).warn("resubscribe failed; retrying in %.2fs", d)
                await asyncio.sleep(d)

    async def _iter(self) -> AsyncIterator[Delivery]:
        while True:
            d = await self._out.get()
            if d is None:
                return
            if d.stale:
                continue  # its channel died before we got to it; the broker requeued it
            yield d

    def get_nowait(self) -> Delivery | None:
        """The next delivery already received (None: shutdown); raises
        ``asyncio.QueueEmpty`` when none is waiting."""
        while True:
            d = self._out.get_nowait()
            if d is None or not d.stale:
                return d

    async def get(self, timeout: float | None = None) -> Delivery | None:
        """Pull the next delivery (None on shutdown / timeout)."""
        try:
            while True:
                d = await asyncio.wait_for(self._out.get(), timeout)
                if d is None or not d.stale:
                    return d
        except asyncio.TimeoutError:
            return None

    # ------------------------------------------------------------ publish
    async def _publisher(self) -> Channel:
        if self._pub is None or self._pub.is_closed:
            ch = await self._channel(qos=False)
            await ch.confirm_select()
            self._pub = ch
        return self._pub

    async def _ensure_publish_topology(self, topic: str) -> None:
        """Best-effort declare of the publish exchange (+ shard queues) once per
        connection, on a scratch channel.  A 403/406 means the topology belongs
        to someone else (a converter that declared quorum queues, a user with
        write-only permission): remember the topic and publish without
        declaring, exactly as the reference always did (``client.go:224``)."""
        if not self.declare_publish or topic in self._declared_pub or topic in self.external_topics:
            return
        ch = await self._channel(qos=False)
        try:
            await ch.exchange_declare(topic, "direct", durable=True)
            if self.declare_publish_queues:
                for i in range(self.num_shard_queues):
                    q = self.get_rk(topic, i)
                    if q in self.external_queues:
                        continue
                    await ch.queue_declare(q, durable=True)
                    await ch.queue_bind(q, topic, q)
        except ChannelClosed as e:
            if not _refused(e):
                raise
            self.external_topics.add(topic)
            log.with_fields(topic=topic, error=str(e)).warn(
                "publish topology is not ours; publishing without declaring it")
            return
        finally:
            if not ch.is_closed:
                await ch.close()
        self._declared_pub.add(topic)

    def _next_rk(self, topic: str) -> str:
        it = self._rk_index.get(topic)
        if it is None:
            it = self._rk_index[topic] = itertools.cycle(range(self.num_shard_queues))
        return self.get_rk(topic, next(it))

    async def publish(self, topic: str, body: bytes, *, headers: dict | None = None,
                      max_attempts: int = 8) -> None:
        """Publish a persistent octet-stream message round-robin over the topic's shards
        and wait for the broker's confirm (retries with backoff)."""
        rk = self._next_rk(topic)
        props = Properties(content_type="application/octet-stream", delivery_mode=codec.PERSISTENT,
                           headers=headers)
        await self._publish_retry(topic, rk, body, props, max_attempts, declare=True)

    async def publish_raw(self, exchange: str, routing_key: str, body: bytes, props: Properties,
                          max_attempts: int = 8) -> None:
        await self._publish_retry(exchange, routing_key, body, props, max_attempts, declare=False)

    def delay_queue_name(self, routing_key: str, delay: float) -> str:
        return f"{routing_key}.retry.{int(round(delay * 1000))}ms"

    async def _ensure_delay_queue(self, exchange: str, routing_key: str, delay: float) -> str:
        """Durable queue ``<rk>.retry.<ms>ms``: ``x-message-ttl`` = delay, expired
        messages dead-letter back to ``exchange`` with the original routing key.
        One queue per (shard, delay) so every message in it has the same TTL
        (RabbitMQ only expires at the queue head).  Declared on a scratch
        channel; a refusal is remembered and raised as :class:`DelayUnavailable`."""
        name = self.delay_queue_name(routing_key, delay)
        if name in self._declared_delay:
            return name
        if name in self._refused_delay:
            raise DelayUnavailable(f"delay queue '{name}' was refused")
        ch = await self._channel(qos=False)
        try:
            await ch.queue_declare(name, durable=True, arguments={
                "x-message-ttl": int(round(delay * 1000)), "x-dead-letter-exchange": exchange,
                "x-dead-letter-routing-key": routing_key})
        except ChannelClosed as e:
            if not _refused(e):
                raise
            self._refused_delay.add(name)
            raise DelayUnavailable(str(e)) from e
        finally:
            if not ch.is_closed:
                await ch.close()
        self._declared_delay.add(name)
        return name

    async def publish_delayed(self, exchange: str, routing_key: str, body: bytes, props: Properties, delay: float,
                              max_attempts: int = 8) -> None:
        """Confirmed publish that reaches ``exchange``/``routing_key`` after ``delay``
        seconds, through the broker.  :class:`DelayUnavailable` if the broker
        refuses the delay queue (the caller waits in-process instead)."""
        pol = ExponentialBackoff(initial=0.05, multiplier=2.0, max_interval=5.0, max_elapsed=None)
        for attempt in range(1, max_attempts + 1):
            try:
                q = await self._ensure_delay_queue(exchange, routing_key, delay)
                async with self._pub_lock:
                    ch = await self._publisher()
                    confirm = await ch.basic_publish("", q, body, props, mandatory=self.mandatory,
                                                     wait_confirm=False)
                if confirm is not None:
                    try:
                        await confirm
                    except ChannelClosed as e:
                        if _refused(e):            # no write on the default exchange
                            self._refused_delay.add(q)
                            raise DelayUnavailable(str(e)) from e
                        raise
                return
            except DelayUnavailable:
                raise
            except PublishReturned as e:
                # the delay queue was deleted after it was declared: without mandatory the
                # retry copy vanished and the caller acked the original (a lost job)
                self._declared_delay.discard(q)
                if attempt == max_attempts or self._closing:
                    raise
                log.with_fields(queue=q, error=str(e)).warn("delay queue gone; declaring it again")
            except (AMQPError, ConnectionError, OSError) as e:
                if attempt == max_attempts or self._closing:
                    raise
                d = pol.next_delay() or 0.0
                log.with_fields(error=str(e), attempt=attempt).warn("delayed publish failed; retrying in %.2fs", d)
                await asyncio.sleep(d)

    def park(self, d: Delivery, props: Properties, delay: float, on_done=None) -> None:
        """The reference's ``Error()`` (``delivery.go:66-84``) without holding the
        job slot: a task waits ``delay``, re-publishes the body to the delivery's
        own exchange/routing key with ``props`` (confirmed) and acks.  A crash
        or shutdown meanwhile leaves the delivery unacked, so the broker
        redelivers it: nothing is lost.

        The parked delivery stays unacked, so it would hold its consumer's
        prefetch slot for the whole wait.  Under per-consumer QoS a new
        ``basic.qos`` only applies to consumers started after it, so instead
        of raising the limit the shard's consumer is replaced
        (:meth:`_rotate`): ``basic.cancel`` + ``basic.consume`` on the same
        channel.  The parked delivery stays unacked on the channel (acks by
        delivery tag still work) but no longer counts against the new
        consumer, so the shard keeps delivering.  With the default prefetch 1
        the old consumer held only the parked delivery, so the limit stays
        exact; with prefetch P > 1, deliveries the old consumer still has in
        flight are not counted against the new one until they settle (at most
        P - 1 extra, transiently)."""
        self.parked_total += 1
        d.requeue_props = props
        d.hold()                            # a long park must not sit unacked past consumer_timeout
        self._spawn_bg(self._parked_retry(d, props, delay, on_done))

    # ------------------------------------------------------------ leases
    def _lease_props(self, d: Delivery) -> Properties:
        base = d.requeue_props or d.msg.properties
        hdrs = dict(base.headers or {})
        hdrs.pop("x-death", None)
        hdrs[LEASE_HOLDER] = _HOLDER
        if d.lease_returns:
            hdrs[LEASE_RETURNS] = d.lease_returns
        else:
            hdrs.pop(LEASE_RETURNS, None)
        return dataclasses.replace(base, headers=hdrs, delivery_mode=codec.PERSISTENT, expiration=None)

    @contextlib.asynccontextmanager
    async def _ops(self):
        """A plain channel for lease declares and deletes.  AMQP allows one
        synchronous method in flight per channel, so concurrent jobs take
        channels of their own from a small free list instead of queueing
        behind one (at 20 ms RTT a shared channel capped leasing at ~25
        jobs/s).  A refusal closes a channel; it is not returned."""
        ch = None
        while self._ops_free:
            c = self._ops_free.pop()
            if not c.is_closed and self.conn is not None and c.conn is self.conn:
                ch = c
                break
        if ch is None:
            ch = await self._channel(qos=False)
        try:
            yield ch
        finally:
            if not ch.is_closed and ch.conn is self.conn and len(self._ops_free) < OPS_CHANNELS:
                self._ops_free.append(ch)
            elif not ch.is_closed:
                with contextlib.suppress(AMQPError, ConnectionError, OSError):
                    await ch.close()

    async def _lease_put(self, d: Delivery, lease: Lease) -> str:
        """Declare lease queue number ``lease.n`` and put the job's copy in it
        (confirmed, mandatory).  :class:`LeaseRefused` when the broker will not
        let this user have it (403/406 on the declare, or on the publish into
        the default exchange)."""
        name = f"{d.routing_key}.lease.{lease.token}.{lease.n}"
        ms = max(1, int(round(lease.ttl * 1000)))
        try:
            async with self._ops() as ch:
                # x-expires well past the TTL: the copy dead-letters first, then the empty queue goes
                await ch.queue_declare(name, durable=True, arguments={
                    "x-message-ttl": ms, "x-expires": 2 * ms + 10_000,
                    "x-dead-letter-exchange": d.exchange, "x-dead-letter-routing-key": d.routing_key})
        except ChannelClosed as e:
            if _refused(e):
                raise LeaseRefused(str(e)) from e
            raise
        async with self._pub_lock:
            pub = await self._publisher()
            confirm = await pub.basic_publish("", name, d.body, self._lease_props(d), mandatory=self.mandatory,
                                              wait_confirm=False)
        if confirm is not None:
            try:
                await confirm
            except ChannelClosed as e:
                if _refused(e):
                    with contextlib.suppress(AMQPError, ConnectionError, OSError):
                        await self._lease_drop(name)
                    raise LeaseRefused(str(e)) from e
                raise
        return name

    async def _lease_drop(self, name: str) -> int:
        """Delete a lease queue; returns how many copies were still in it
        (RabbitMQ discards them, it does not dead-letter on delete)."""
        async with self._ops() as ch:
            return await ch.queue_delete(name)

    async def _lease_take(self, d: Delivery, ttl: float) -> bool:
        lease = Lease(secrets.token_hex(6), ttl)
        try:
            lease.queue = await self._lease_put(d, lease)
        except LeaseRefused as e:
            self._lease_refused.add(d.routing_key)
            self.lease_stats["refused"] += 1
            log.with_fields(routing_key=d.routing_key, error=str(e)).warn(
                "the broker refused a lease queue; holding deliveries unacked for the whole job instead (a job "
                "longer than the broker's consumer_timeout will be requeued): grant configure on '<shard>.lease.*'")
            return False
        try:
            if d.msg.channel is None or d.msg.channel.is_closed:
                raise ChannelClosed(0, "delivery channel gone")
            await d.msg.ack()
            self._unhold(d)
        except (AMQPError, ConnectionError, OSError):
            # the broker took the original back already (consumer timeout, channel error):
            # the copy must not come back as a second job
            with contextlib.suppress(AMQPError, ConnectionError, OSError):
                await self._lease_drop(lease.queue)
            return False
        d.lease = lease
        self._leased.add(d)
        self.lease_stats["taken"] += 1
        log.with_fields(queue=lease.queue, ttl_s=ttl).info("job leased: its delivery is acked, the broker holds a copy")
        return True

    async def _lease_renew(self, d: Delivery) -> None:
        """Copy ``n + 1`` first, then delete copy ``n``: there is always a copy.
        If copy ``n`` was gone, the lease had run out (a long broker outage)
        and the job went back to its queue; the new copy is dropped too."""
        lease = d.lease
        assert lease is not None
        old = lease.queue
        lease.n += 1
        try:
            new = await self._lease_put(d, lease)
        except BaseException:
            with contextlib.suppress(BaseException):
                await asyncio.wait_for(self._lease_drop(f"{d.routing_key}.lease.{lease.token}.{lease.n}"), 5.0)
            raise
        lease.queue = new
        if await self._lease_drop(old) == 0:
            lease.lost = True
            self.lease_stats["lost"] += 1
            log.with_fields(queue=old).error("job lease ran out before it was renewed; the job went back to its "
                                             "queue and may run twice")
            with contextlib.suppress(AMQPError, ConnectionError, OSError):
                await self._lease_drop(new)
            self._leased.discard(d)
            return
        lease.renewed_at = time.monotonic()
        self.lease_stats["renewed"] += 1

    async def _lease_release(self, d: Delivery, requeue: bool = False) -> bool:
        """Settle a leased delivery: with ``requeue`` the job goes back to its
        queue now (a graceful shutdown), then the lease copy is deleted.  False
        when the lease had already run out (the job went back on its own)."""
        lease = d.lease
        assert lease is not None
        if lease.lost:
            return False
        if requeue:
            try:
                await self.publish_raw(d.exchange, d.routing_key, d.body, d.requeue_props or d.retry_props(0),
                                       max_attempts=3)
            except Exception as e:  # noqa: BLE001 - the lease copy stays: it comes back when it expires
                log.with_fields(error=str(e), queue=lease.queue).warn("could not requeue a leased job; it comes "
                                                                     "back when its lease runs out")
                return False
            self.lease_stats["requeued"] += 1
        pol = ExponentialBackoff(initial=0.05, max_interval=2.0, max_elapsed=None)
        while True:
            try:
                n = await self._lease_drop(lease.queue)
                break
            except (AMQPError, ConnectionError, OSError) as e:
                if time.monotonic() - lease.renewed_at > lease.ttl or (self._closing and not requeue):
                    n = 0                    # ran out meanwhile: the broker has given the job back
                    break
                d2 = pol.next_delay() or 1.0
                log.with_fields(error=str(e), queue=lease.queue).warn("releasing the job lease failed; retrying")
                await asyncio.sleep(d2)
        if n == 0:
            lease.lost = True
            self.lease_stats["lost"] += 1
            if not requeue:
                log.with_fields(queue=lease.queue).error("job lease had run out; the job went back to its queue")
            return False
        self.lease_stats["released"] += 1
        return True

    async def _hold(self, d: Delivery, after: float, ttl: float) -> None:
        """Take ``d``'s lease after ``after`` s, then renew it every ``ttl / 2``
        until it is settled.  Every step runs under the delivery's settle lock
        and retries outside it, so an ack never waits on an outage."""
        try:
            await asyncio.sleep(after)
            pol = ExponentialBackoff(initial=0.2, max_interval=5.0, max_elapsed=None)
            while True:
                async with d._settle_lock():
                    if d.settled or d.stale or self._closing or d.routing_key in self._lease_refused:
                        return
                    try:
                        if not await self._lease_take(d, ttl):
                            return
                        break
                    except (AMQPError, ConnectionError, OSError) as e:
                        log.with_field("error", str(e)).warn("taking a job lease failed; retrying")
                await asyncio.sleep(pol.next_delay() or 1.0)
            pol.reset()
            wait = ttl / 2
            while True:
                await asyncio.sleep(wait)
                async with d._settle_lock():
                    if d.settled or d.lease is None or d.lease.lost or self._closing:
                        return
                    try:
                        await self._lease_renew(d)
                        wait = ttl / 2
                        pol.reset()
                    except (AMQPError, ConnectionError, OSError) as e:
                        wait = min(ttl / 4, pol.next_delay() or 1.0)
                        log.with_field("error", str(e)).warn("renewing a job lease failed; retrying in %.1fs", wait)
        except asyncio.CancelledError:
            pass

    async def _release_leases(self) -> None:
        """Shutdown: every held delivery stops renewing; a leased one that is
        not settled goes back to its queue at once (not after its TTL)."""
        for d in list(self._holding):
            async with d._settle_lock():
                if d._hold is not None:
                    d._hold.cancel()
            if d.lease is not None and not d.settled:
                with contextlib.suppress(Exception):
                    await asyncio.wait_for(d.nack(requeue=True), 10.0)

    def _unhold(self, d: Delivery) -> None:
        """``d`` no longer counts against its shard consumer's prefetch."""
        sh = self._shard_of(d.msg.channel)
        if sh is not None:
            sh.held.pop(d.msg.delivery_tag, None)

    def _shard_of(self, ch: Channel | None) -> Shard | None:
        for sh in self.shards.values():
            if sh.channel is ch:
                return sh
        return None

    async def _rotate(self, shard: Shard, tag: str) -> bool:
        """Replace ``shard``'s consumer ``tag`` with a fresh one on the same
        channel (its per-consumer unacked count starts at 0).  False if the
        consumer is already gone or replaced."""
        async with shard.lock:
            ch = shard.channel
            if ch is None or ch.is_closed or not shard.active or shard.tag != tag or self._closing:
                return False
            cb = shard.on_msg
            await ch.basic_cancel(tag)
            new = await ch.basic_consume(shard.queue, cb, no_ack=False)
            shard.set_active(ch, new, cb)
            shard.rotations += 1
            return True

    async def set_live_prefetch(self, prefetch: int) -> None:
        """Change every shard consumer's prefetch while consuming: per-consumer
        ``basic.qos`` applies only to consumers started after it, so each
        shard's consumer is re-subscribed on its channel (its unacked
        deliveries stay ackable there).  Channels opened later (a reconnect)
        use the new value too."""
        self.prefetch = prefetch
        for sh in list(self.shards.values()):
            async with sh.lock:
                ch = sh.channel
                if ch is None or ch.is_closed or self._closing:
                    continue
                await ch.basic_qos(prefetch, 0, False)
                if not sh.active or sh.paused or sh.on_msg is None:
                    continue                 # resume() / reopen consume with the new qos
                cb = sh.on_msg
                await ch.basic_cancel(sh.tag)
                new = await ch.basic_consume(sh.queue, cb, no_ack=False)
                sh.set_active(ch, new, cb)

    # ------------------------------------------------------------ hand-back
    async def pause(self) -> int:
        """Stop taking deliveries and give back the ones buffered here.

        With prefetch per shard consumer, a worker busy with a long job holds
        one more delivery per other shard.  That delivery waits behind the job,
        maybe for hours of a torrent, while other workers sit idle, and
        RabbitMQ's ``consumer_timeout`` runs for it too.  The reference worked
        the same way (``client.go:360-373``, one goroutine per worker).  This
        method cancels every shard consumer, so no more deliveries arrive, and
        keeps the channels open, so deliveries still unacked can be acked.
        Each buffered delivery is then re-published to its own exchange and
        routing key (confirmed; a fresh message, so no redelivery count) and
        the original acked.  If the re-publish fails, the delivery is
        nack-requeued.  Returns how many were handed back; :meth:`resume`
        consumes again."""
        if self.paused:
            return 0
        self.paused = True
        for sh in list(self.shards.values()):
            async with sh.lock:
                ch = sh.channel
                if not sh.active or ch is None or ch.is_closed:
                    continue
                try:
                    # deliveries the broker sent before its cancel-ok are in _out when this returns
                    await ch.basic_cancel(sh.tag)
                except AMQPError as e:
                    log.with_fields(queue=sh.queue, error=str(e)).warn("pausing the consumer failed")
                    continue
                sh.set_inactive()
                sh.paused = True
        held: list[Delivery] = []
        stop = False
        while not self._out.empty():
            d = self._out.get_nowait()
            if d is None:
                stop = True                 # the shutdown sentinel goes back after them
                continue
            held.append(d)
        if stop:
            self._out.put_nowait(None)
        n = 0
        for d in held:
            if d.stale:
                continue                    # its channel died: the broker requeued it already
            props = d.msg.properties
            if d.msg.redelivered:
                props = dataclasses.replace(props, headers={**(props.headers or {}), REDELIVERED: 1})
            try:
                await self.publish_raw(d.exchange, d.routing_key, d.body, props, max_attempts=3)
                await d.ack()
                n += 1
            except Exception as e:  # noqa: BLE001 - the original is still unacked: requeue it
                log.with_field("error", str(e)).warn("hand-back re-publish failed; requeueing the delivery")
                with contextlib.suppress(Exception):
                    await d.nack(requeue=True)
        self.handed_back += n
        if n:
            log.with_fields(deliveries=n).info("busy with a long job: handed buffered deliveries back to the broker")
        return n

    async def resume(self) -> None:
        """Consume again on every shard :meth:`pause` stopped."""
        if not self.paused:
            return
        self.paused = False
        for sh in list(self.shards.values()):
            async with sh.lock:
                ch = sh.channel
                if sh.active or not sh.paused or ch is None or ch.is_closed or sh.on_msg is None:
                    sh.paused = False
                    continue
                try:
                    tag = await ch.basic_consume(sh.queue, sh.on_msg, no_ack=False)
                except AMQPError as e:
                    sh.paused = False        # now a real outage: health and the reopen paths see it
                    log.with_fields(queue=sh.queue, error=str(e)).warn("resuming the consumer failed")
                    continue
                sh.set_active(ch, tag, sh.on_msg)

    async def _parked_retry(self, d: Delivery, props: Properties, delay: float, on_done=None) -> None:
        self._parked += 1
        try:
            shard = self._shard_of(d.msg.channel) if d.lease is None else None
            if shard is not None and d.msg.consumer_tag:
                try:
                    await self._rotate(shard, d.msg.consumer_tag)
                except AMQPError as e:       # the channel died: the broker requeued the delivery
                    log.with_fields(queue=shard.queue, error=str(e)).warn("consumer re-subscribe failed")
            await asyncio.sleep(delay)
            if d.stale:
                return                      # its channel died: the broker requeued it already
            await self.publish_raw(d.exchange, d.routing_key, d.body, props)
            await d.ack()
            log.with_fields(routing_key=d.routing_key, retries=(props.headers or {}).get("X-Retries")).info(
                "parked delivery re-published")
        except asyncio.CancelledError:
            raise
        except Exception as e:  # noqa: BLE001 - the original is still unacked: give it back once
            log.with_field("error", str(e)).error("parked re-publish failed; requeueing the delivery")
            with contextlib.suppress(Exception):
                await d.nack(requeue=True)
        finally:
            self._parked -= 1
            if on_done is not None:
                on_done()

    @property
    def parked(self) -> int:
        """Deliveries currently waiting in-process (:meth:`park`)."""
        return self._parked

    # ------------------------------------------------------------ health
    async def ready_counts(self, topic: str) -> dict[str, int]:
        """Ready (undelivered) messages on each of ``topic``'s shard queues, by
        passive declare on a scratch channel (no permission needed)."""
        ch = await self._channel(qos=False)
        try:
            out = {}
            for i in range(self.num_shard_queues):
                q = self.get_rk(topic, i)
                _q, count, _consumers = await ch.queue_declare(q, passive=True)
                out[q] = count
            return out
        finally:
            if not ch.is_closed:
                await ch.close()

    async def ready_count(self, topic: str) -> int:
        return sum((await self.ready_counts(topic)).values())

    def health(self, max_down_s: float) -> tuple[bool, list[str]]:
        """(healthy, reasons).  Unhealthy once the connection has been down for
        more than ``max_down_s`` (the supervisor is still reconnecting), or once
        any shard of a consumed topic has had no consumer for that long (a
        consumer stuck in its re-subscribe / reopen retry loop, a queue that
        was deleted or that this user may no longer read)."""
        now = time.monotonic()
        why: list[str] = []
        if self._closing:
            why.append("closing")
        if self.lost_since is not None and now - self.lost_since > max_down_s:
            why.append(f"broker connection down for {now - self.lost_since:.0f}s")
        for q, sh in sorted(self.shards.items()):
            down = sh.down_for(now)
            if down > max_down_s:
                why.append(f"no consumer on {q} for {down:.0f}s")
        return (not why, why)

    async def _publish_retry(self, exchange: str, rk: str, body: bytes, props: Properties, max_attempts: int,
                             declare: bool) -> None:
        pol = ExponentialBackoff(initial=0.05, multiplier=2.0, max_interval=5.0, max_elapsed=None)
        for attempt in range(1, max_attempts + 1):
            try:
                async with self._pub_lock:
                    if declare:
                        await self._ensure_publish_topology(exchange)
                    ch = await self._publisher()
                    # frames leave in order under the lock; the confirm is awaited outside
                    # it, so concurrent jobs' publishes share broker round trips
                    t_pub = time.monotonic()
                    confirm = await ch.basic_publish(exchange, rk, body, props, mandatory=self.mandatory,
                                                     wait_confirm=False)
                if confirm is not None:
                    await confirm
                    dt = time.monotonic() - t_pub
                    e = self.confirm_ewma
                    self.confirm_ewma = dt if e is None else e + 0.2 * (dt - e)
                log.info("published message on topic %s", exchange)
                return
            except PublishReturned as e:
                # confirmed but routed nowhere: RabbitMQ would have dropped it silently (and
                # so did the reference's publish).  Re-declare the shard queue and binding
                # (when the topology is ours) and publish again; a topology that stays
                # unroutable fails the publish, so the job is retried, never lost
                self.returned += 1
                self._declared_pub.discard(exchange)
                if attempt == max_attempts or self._closing:
                    log.with_fields(error=str(e)).error("publish unroutable; giving up")
                    raise
                d = pol.next_delay() or 0.0
                log.with_fields(error=str(e), attempt=attempt).warn("publish unroutable; retrying in %.2fs", d)
                await asyncio.sleep(d)
            except (AMQPError, ConnectionError, OSError) as e:
                if attempt == max_attempts or self._closing or self._permanent(exchange, e):
                    raise
                if isinstance(e, ChannelClosed) and e.code == codec.NOT_FOUND:
                    self._declared_pub.discard(exchange)   # deleted since we declared it: declare again
                d = pol.next_delay() or 0.0
                log.with_fields(error=str(e), attempt=attempt).warn("publish failed; retrying in %.2fs", d)
                await asyncio.sleep(d)

    def _permanent(self, exchange: str, e: BaseException) -> bool:
        """Publish failures a retry cannot fix: no write permission on the
        exchange, or an exchange that is missing and that we may not declare."""
        if not isinstance(e, ChannelClosed):
            return False
        return e.code == codec.ACCESS_REFUSED or (e.code == codec.NOT_FOUND and exchange in self.external_topics)

    # ------------------------------------------------------------ shutdown
    async def close(self) -> None:
        """Stop consuming and close the connection (``Done`` semantics).
        Leased jobs still running go back to their queues first."""
        if self._holding and self.connected:
            await self._release_leases()
        self._closing = True
        for d in list(self._holding):
            if d._hold is not None:
                d._hold.cancel()
        self._lost.set()
        if self._supervisor is not None:
            self._supervisor.cancel()
            with contextlib.suppress(BaseException):
                await self._supervisor
        for t in list(self._bg):
            t.cancel()
            with contextlib.suppress(BaseException):
                await t
        if self.conn is not None:
            for ch in self._consumer_chans:
                with contextlib.suppress(Exception):
                    if not ch.is_closed:
                        await asyncio.wait_for(ch.close(), 2)
            with contextlib.suppress(Exception):
                await self.conn.close()
        self._out.put_nowait(None)

    @property
    def connected(self) -> bool:
        return self.conn is not None and not self.conn.is_closed


__all__ = ["Client", "Delivery", "DeliveryMetadata", "ConsumeError", "ConnectionClosed", "DelayUnavailable"]
