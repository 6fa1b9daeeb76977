"""Job producer and ``v1.convert`` counter for the benches, in a process of
its own.

It stands in for the other tritonmedia services on each side of the worker:
the one that publishes ``v1.download`` jobs and the one that consumes
``v1.convert``.  The bench's timed region measures workers only when those
run elsewhere.  Before, rank 0's worker process also hosted them, so rank 0's
event loop published every job, decoded every ``Convert`` and acked it,
alongside its own worker.  Rank 0 starts this process and drives it with JSON
lines:

    python -m tritondl_testkit.bench_producer --broker URL --origins U1,U2 --size BYTES [--tag T]
        stdout  {"ready": true}
        stdin   {"cmd": "run", "n": N}   publish N jobs (pipelined confirms) and
                                         wait until N new converts arrived
        stdout  {"done": N, "elapsed": s, "cpu": {"producer": s, "broker": s}}
        stdin   EOF                      exit

Each ``Convert`` is checked on the way in (the job's media id, exactly once).
Dead-lettered jobs (``v1.download.dead``) end a run at once with an error
naming the failed stage (the bench runs with ``max_retries=0``), instead of
waiting out the timeout.  ``--variants R``: job ``i`` fetches payload
variant ``i % R`` (:mod:`tritondl_testkit.fakes.payload`).
``--broker-pid`` names the broker process whose CPU time the reply reports
(psutil), so a run can tell when the single-process fake broker, not the
workers, is the bottleneck.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import resource
import sys
import time

from tritondl.amqp.codec import Properties
from tritondl.amqp.connection import Connection
from tritondl.models import Convert, Download, Media, SourceType


def _cpu_self() -> float:
    ru = resource.getrusage(resource.RUSAGE_SELF)
    return ru.ru_utime + ru.ru_stime


def _cpu_of(pid: int) -> float:
    if not pid:
        return 0.0
    try:
        import psutil
        t = psutil.Process(pid).cpu_times()
        return t.user + t.system
    except Exception:  # noqa: BLE001 - reporting only
        return 0.0


class Producer:
    def __init__(self, broker: str, origins: list[str], size: int, tag: str = "p", shards: int = 2,
                 variants: int = 0) -> None:
        self.broker, self.origins, self.size, self.tag, self.shards = broker, origins, size, tag, shards
        self.variants = variants
        self.dead: list[str] = []
        self.conn: Connection | None = None
        self.n = 0
        self.seen: set[str] = set()
        self.dups = 0
        self._target = 0
        self._got = asyncio.Event()

    async def start(self) -> "Producer":
        self.conn = await Connection.open(self.broker, heartbeat=0)
        self.pch = await self.conn.channel()
        await self.pch.confirm_select()
        self.cch = await self.conn.channel()
        await self.pch.exchange_declare("v1.download", "direct", durable=True)
        for i in range(self.shards):
            await self.pch.queue_declare(f"v1.download-{i}", durable=True)
            await self.pch.queue_bind(f"v1.download-{i}", "v1.download", f"v1.download-{i}")
            await self.cch.queue_declare(f"v1.convert-{i}", durable=True)
            await self.cch.basic_consume(f"v1.convert-{i}", self._on_convert)
        await self.cch.exchange_declare("v1.download.dead", "direct", durable=True)
        for i in range(self.shards):
            q = f"v1.download.dead-{i}"
            await self.cch.queue_declare(q, durable=True)
            await self.cch.queue_bind(q, "v1.download.dead", q)
            await self.cch.basic_consume(q, self._on_dead)
        return self

    def _on_dead(self, m) -> None:
        h = m.properties.headers or {}
        self.dead.append(f"{h.get('X-Failed-Stage', '?')}: {h.get('X-Error', '?')}")
        asyncio.ensure_future(m.ack())
        self._got.set()

    def _on_convert(self, m) -> None:
        c = Convert.decode(m.body)
        mid = c.media.id if c.media is not None else ""
        if mid in self.seen or not mid.startswith(f"bench-{self.tag}-"):
            self.dups += 1
        else:
            self.seen.add(mid)
        asyncio.ensure_future(m.ack())
        if len(self.seen) >= self._target:
            self._got.set()

    def job_body(self, i: int) -> tuple[str, bytes]:
        mid = f"bench-{self.tag}-{i}"
        origin = self.origins[i % len(self.origins)]
        name = f"movie-{i}-v{i % self.variants}.mkv" if self.variants else f"movie-{i}.mkv"
        url = f"{origin}/synthetic/{self.size}/{name}"
        d = Download(created_at="now", media=Media(id=mid, name=f"movie {i}", source=SourceType.HTTP,
                                                      source_uri=url))
        return mid, d.encode()

    async def submit(self, n: int) -> None:
        """Publish with confirms pipelined (up to 256 outstanding): one broker
        round trip per batch, not per job."""
        pending: list[asyncio.Future] = []
        for _ in range(n):
            i = self.n
            self.n += 1
            _mid, body = self.job_body(i)
            fut = await self.pch.basic_publish("v1.download", f"v1.download-{i % self.shards}", body,
                                               Properties(delivery_mode=2, content_type="application/octet-stream"),
                                               wait_confirm=False)
            if fut is not None:
                pending.append(fut)
            if len(pending) >= 256:
                await asyncio.gather(*pending)
                pending.clear()
        if pending:
            await asyncio.gather(*pending)

    async def run(self, n: int, timeout: float = 600) -> float:
        base = len(self.seen)
        self._target = base + n
        self._got.clear()
        t0 = time.perf_counter()
        await self.submit(n)
        deadline = time.monotonic() + timeout
        while len(self.seen) < self._target and not self.dead:
            self._got.clear()
            try:
                await asyncio.wait_for(self._got.wait(), max(0.0, deadline - time.monotonic()))
            except asyncio.TimeoutError:
                raise TimeoutError(f"only {len(self.seen) - base}/{n} converts") from None
        if self.dead:
            raise RuntimeError(f"{len(self.dead)} jobs dead-lettered, first: {self.dead[0]}")
        return time.perf_counter() - t0

    async def close(self) -> None:
        if self.conn is not None:
            await self.conn.close()


async def _amain(a: argparse.Namespace) -> None:
    p = await Producer(a.broker, a.origins.split(","), a.size, a.tag, variants=a.variants).start()
    loop = asyncio.get_running_loop()
    reader = asyncio.StreamReader()
    await loop.connect_read_pipe(lambda: asyncio.StreamReaderProtocol(reader), sys.stdin)
    print(json.dumps({"ready": True}), flush=True)
    try:
        while True:
            line = await reader.readline()
            if not line:
                return
            cmd = json.loads(line)
            if cmd.get("cmd") != "run":
                continue
            c0, b0 = _cpu_self(), _cpu_of(a.broker_pid)
            try:
                dt = await p.run(int(cmd["n"]), float(cmd.get("timeout", 600)))
                out = {"done": int(cmd["n"]), "elapsed": dt, "dups": p.dups,
                       "cpu": {"producer": _cpu_self() - c0, "broker": _cpu_of(a.broker_pid) - b0}}
            except Exception as e:  # noqa: BLE001 - reported to the driver
                out = {"error": str(e)}
            print(json.dumps(out), flush=True)
    finally:
        await p.close()


def main() -> None:
    from tritondl.parallel.topology import pin_from_env
    pin_from_env()
    ap = argparse.ArgumentParser()
    ap.add_argument("--broker", required=True)
    ap.add_argument("--origins", required=True, help="comma-separated origin base URLs (jobs round-robin)")
    ap.add_argument("--size", type=int, required=True)
    ap.add_argument("--tag", default="p")
    ap.add_argument("--broker-pid", type=int, default=0)
    ap.add_argument("--variants", type=int, default=0, help="payload variants (job i fetches i %% R)")
    asyncio.run(_amain(ap.parse_args()))


if __name__ == "__main__":
    main()
