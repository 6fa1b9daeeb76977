"""Multi-process worker pool with failure detection and restart.

Each worker is a full ingest service process (``python -m tritondl``)
consuming the same sharded queues — competing consumers, the reference's
scale-out model — so jobs spread across workers and a
crashed worker's unacked job is redelivered by the broker to a survivor.

The supervisor:

* starts N workers with per-worker env (rank, GPU, BT port, CPU affinity);
* detects exits (any non-zero exit or signal death) and restarts the
  worker with exponential backoff; a worker that crash-loops
  (``max_restarts`` within ``restart_window``) is given up on;
* on SIGTERM/SIGINT forwards SIGTERM to every worker, waits ``grace`` s,
  then SIGKILLs stragglers — by PID, never by name;
* fails loudly: once fewer than ``min_workers`` workers are left (default
  1: every worker given up), it stops the rest and exits non-zero so the
  orchestrator restarts the pod — the reference's ``log.Fatal`` exits
  (``cmd/downloader/downloader.go:64,70,83,92,97``).  ``/healthz`` on
  ``--health-addr`` answers 503 while any worker is given up, or while any
  running worker's own ``/healthz`` does (a worker whose shard consumer or
  broker connection has been down too long, or that sits idle on a
  backlog: :meth:`tritondl.service.Service.health`).  Each worker serves
  its ``/healthz`` on loopback port ``health port + 1 + rank``, or where
  ``TRITONDL_METRICS_ADDR`` says (set for all workers, worker ``r`` serves
  its port + ``r``); the pool polls the address each worker serves.
  ``/metrics`` carries live / given-up / unhealthy / restart counts.
"""

from __future__ import annotations

import asyncio
import contextlib
import os
import signal
import sys
import time
from dataclasses import dataclass, field

from ..utils.log import log
from ..utils.metrics import Metrics, serve_metrics
from .topology import WorkerSpec, plan


@dataclass
class _Worker:
    spec: WorkerSpec
    proc: asyncio.subprocess.Process | None = None
    restarts: list[float] = field(default_factory=list)
    given_up: bool = False
    started_at: float = 0.0
    health_addr: tuple[str, int] | None = None   # where this worker serves /healthz (None: nowhere known)


class WorkerPool:
    def __init__(self, specs: list[WorkerSpec], *, argv: list[str] | None = None, env: dict | None = None,
                 max_restarts: int = 5, restart_window: float = 60.0, grace: float = 30.0,
                 backoff_initial: float = 0.5, backoff_max: float = 30.0, cwd: str | None = None,
                 module: str = "tritondl", worker_env=None, min_workers: int = 1,
                 health_addr: str = "", worker_health_base: int = 0, worker_health_grace: float = 60.0) -> None:
        """``worker_env(rank) -> dict``: extra env for one worker (e.g. its
        nearest S3 node).  ``worker_health_base``: worker ``r`` serves its
        ``/healthz`` on ``127.0.0.1:base+r`` (default: the pool's health port
        + 1); a worker whose endpoint does not answer within
        ``worker_health_grace`` s of its start counts as unhealthy."""
        self.workers = [_Worker(s) for s in specs]
        self.argv = argv or []
        self.env = env or {}
        self.worker_env = worker_env
        self.max_restarts = max_restarts
        self.restart_window = restart_window
        self.grace = grace
        self.backoff_initial = backoff_initial
        self.backoff_max = backoff_max
        self.cwd = cwd
        self.module = module
        self.min_workers = max(0, min(min_workers, len(self.workers)))
        self.health_addr = health_addr
        if health_addr and not worker_health_base:
            worker_health_base = int(health_addr.rpartition(":")[2]) + 1
        self.worker_health_base = worker_health_base
        self.worker_health_grace = worker_health_grace
        self.metrics = Metrics()
        self._stopping = False
        self._tasks: list[asyncio.Task] = []
        self._failed: asyncio.Event | None = None
        self._health_runner = None
        self.exits: list[tuple[int, int | None]] = []   # (rank, returncode)

    @property
    def live(self) -> int:
        """Workers not given up on (running, or waiting out a restart backoff)."""
        return sum(1 for w in self.workers if not w.given_up)

    @property
    def healthy(self) -> bool:
        """The pool's own view (no worker given up); :meth:`health` adds the workers'."""
        return not any(w.given_up for w in self.workers) and not self._stopping

    def _gauges(self) -> None:
        self.metrics.set("pool_workers_live", self.live)
        self.metrics.set("pool_workers_given_up", len(self.workers) - self.live)

    def _health_port(self, w: _Worker) -> int:
        return self.worker_health_base + w.spec.rank if self.worker_health_base else 0

    @staticmethod
    def _probe_addr(metrics_addr: str) -> tuple[str, int] | None:
        """The address to poll for a worker serving ``host:port``: a wildcard
        host is polled on loopback; None if the value is not host:port."""
        host, _, port = metrics_addr.strip().rpartition(":")
        try:
            p = int(port)
        except ValueError:
            return None
        if not 0 < p < 65536:
            return None
        host = host.strip("[]")
        if host in ("", "0.0.0.0"):
            host = "127.0.0.1"
        elif host == "::":
            host = "::1"
        return host, p

    async def _worker_health(self, w: _Worker) -> str:
        """'' if worker ``w`` is healthy (or still within its start-up grace,
        or between restarts), else why not.  Polled where the worker actually
        serves its ``/healthz`` (its TRITONDL_METRICS_ADDR, the pool's
        ``base + rank`` or an operator's own); a worker with no metrics
        address is not polled."""
        if w.health_addr is None or w.proc is None or w.proc.returncode is not None:
            return ""
        host, port = w.health_addr
        young = time.monotonic() - w.started_at < self.worker_health_grace
        try:
            r, wr = await asyncio.wait_for(asyncio.open_connection(host, port), 2.0)
            try:
                wr.write(b"GET /healthz HTTP/1.0\r\nHost: localhost\r\n\r\n")
                data = await asyncio.wait_for(r.read(1 << 16), 3.0)
            finally:
                wr.close()
            code = int(data.split(b" ", 2)[1])
        except (OSError, asyncio.TimeoutError, ValueError, IndexError) as e:
            return "" if young else f"worker {w.spec.rank}: /healthz unreachable ({e.__class__.__name__})"
        if code == 200:
            return ""
        body = data.split(b"\r\n\r\n", 1)[-1].decode(errors="replace").strip().replace("\n", "; ")
        return f"worker {w.spec.rank}: {body}"

    async def health(self) -> tuple[bool, list[str]]:
        """The pool's ``/healthz``: given-up workers, then every running
        worker's own ``/healthz``."""
        why = [f"worker {w.spec.rank}: given up (crash-looping)" for w in self.workers if w.given_up]
        if self._stopping:
            why.append("stopping")
        polled = await asyncio.gather(*(self._worker_health(w) for w in self.workers if not w.given_up))
        bad = [x for x in polled if x]
        self.metrics.set("pool_workers_unhealthy", len(bad))
        return not (why or bad), why + bad

    async def _spawn(self, w: _Worker) -> None:
        env = dict(os.environ)
        env.update(self.env)
        env.update(w.spec.env())
        per_worker = self.worker_env(w.spec.rank) if self.worker_env is not None else {}
        env.update(per_worker)
        addr = env.get("TRITONDL_METRICS_ADDR", "")
        if not addr and self._health_port(w):
            addr = f"127.0.0.1:{self._health_port(w)}"
        elif addr and "TRITONDL_METRICS_ADDR" not in per_worker and len(self.workers) > 1:
            # one address for every worker (the pool's own environment): they cannot all bind
            # it, so worker r serves port + r
            host, _, port = addr.rpartition(":")
            if port.isdigit():
                addr = f"{host}:{int(port) + w.spec.rank}"
        if addr:
            env["TRITONDL_METRICS_ADDR"] = addr
        w.health_addr = self._probe_addr(addr) if addr else None
        if w.spec.cpus and "TRITONDL_CPUS" not in self.env:
            # the worker pins itself first thing (service.main, TRITONDL_CPUS): no
            # preexec_fn in this threaded supervisor
            env["TRITONDL_CPUS"] = ",".join(map(str, w.spec.cpus))
        w.proc = await asyncio.create_subprocess_exec(sys.executable, "-m", self.module, *self.argv, env=env,
                                                      cwd=self.cwd)
        w.started_at = time.monotonic()
        log.with_fields(rank=w.spec.rank, pid=w.proc.pid, gpu=w.spec.gpu).info("worker started")

    async def _watch(self, w: _Worker) -> None:
        delay = self.backoff_initial
        while not self._stopping:
            await self._spawn(w)
            assert w.proc is not None
            rc = await w.proc.wait()
            self.exits.append((w.spec.rank, rc))
            if self._stopping:
                return
            now = time.monotonic()
            if now - w.started_at > self.restart_window:
                delay = self.backoff_initial  # it ran healthily for a while
            w.restarts = [t for t in w.restarts if now - t < self.restart_window] + [now]
            self.metrics.inc("pool_worker_restarts", rank=str(w.spec.rank))
            if len(w.restarts) > self.max_restarts:
                w.given_up = True
                self._gauges()
                log.with_fields(rank=w.spec.rank, rc=rc, live=self.live).error(
                    "worker is crash-looping; giving up on it")
                if self.live < self.min_workers and self._failed is not None:
                    log.with_fields(live=self.live, min_workers=self.min_workers).error(
                        "fatal: too few workers left; stopping the pool")
                    self._failed.set()
                return
            log.with_fields(rank=w.spec.rank, rc=rc, restart_in=round(delay, 2)).warn("worker died; restarting")
            await asyncio.sleep(delay)
            delay = min(delay * 2, self.backoff_max)

    async def start(self) -> None:
        self._failed = asyncio.Event()
        self._gauges()
        if self.health_addr:
            self._health_runner = await serve_metrics(self.metrics, self.health_addr, health=self.health)
        for w in self.workers:
            self._tasks.append(asyncio.ensure_future(self._watch(w)))
        # wait until every worker has a process
        for _ in range(200):
            if all(w.proc is not None for w in self.workers):
                break
            await asyncio.sleep(0.01)

    def pids(self) -> list[int]:
        return [w.proc.pid for w in self.workers if w.proc is not None and w.proc.returncode is None]

    async def stop(self) -> None:
        self._stopping = True
        procs = [w.proc for w in self.workers if w.proc is not None and w.proc.returncode is None]
        for p in procs:
            with contextlib.suppress(ProcessLookupError):
                p.send_signal(signal.SIGTERM)
        try:
            await asyncio.wait_for(asyncio.gather(*(p.wait() for p in procs)), self.grace)
        except asyncio.TimeoutError:
            for p in procs:
                if p.returncode is None:
                    with contextlib.suppress(ProcessLookupError):
                        p.kill()
            await asyncio.gather(*(p.wait() for p in procs))
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            with contextlib.suppress(BaseException):
                await t
        if self._health_runner is not None:
            await self._health_runner.cleanup()
            self._health_runner = None

    async def run_until_signalled(self) -> int:
        """Run until a signal (returns 0) or until fewer than ``min_workers``
        workers are left (returns 1: the process should exit non-zero)."""
        loop = asyncio.get_running_loop()
        stop = asyncio.Event()
        for s in (signal.SIGINT, signal.SIGTERM, signal.SIGHUP):
            with contextlib.suppress(NotImplementedError, RuntimeError):
                loop.add_signal_handler(s, stop.set)
        await self.start()
        assert self._failed is not None
        sig = asyncio.ensure_future(stop.wait())
        bad = asyncio.ensure_future(self._failed.wait())
        await asyncio.wait({sig, bad}, return_when=asyncio.FIRST_COMPLETED)
        failed = self._failed.is_set()
        for t in (sig, bad):
            t.cancel()
        await self.stop()
        return 1 if failed else 0


def main(argv: list[str] | None = None) -> int:
    import argparse
    ap = argparse.ArgumentParser(prog="python -m tritondl.parallel",
                                 description="run N competing ingest workers on this node")
    ap.add_argument("--workers", type=int, default=None, help="default: one per GPU (or per 2 CPUs)")
    ap.add_argument("--base-port", type=int, default=0, help="BitTorrent listen port of worker 0 (+rank)")
    ap.add_argument("--grace", type=float, default=30.0)
    ap.add_argument("--min-workers", type=int, default=1,
                    help="exit non-zero once fewer workers than this are left (crash-looping ones are given up)")
    ap.add_argument("--health-addr", default="", help="host:port for the pool's /healthz and /metrics")
    ap.add_argument("--worker-health-base", type=int, default=0,
                    help="worker r serves its own /healthz on 127.0.0.1:BASE+r, which the pool's /healthz polls "
                         "(default: the --health-addr port + 1; unless TRITONDL_METRICS_ADDR is set)")
    ap.add_argument("--worker-health-grace", type=float, default=60.0,
                    help="seconds after a worker starts before an unreachable /healthz counts against it")
    ap.add_argument("--max-restarts", type=int, default=5, help="restarts within --restart-window before giving up")
    ap.add_argument("--restart-window", type=float, default=60.0)
    a, rest = ap.parse_known_args(argv)
    pool = WorkerPool(plan(a.workers, base_port=a.base_port), argv=rest, grace=a.grace,
                      min_workers=a.min_workers, health_addr=a.health_addr, max_restarts=a.max_restarts,
                      restart_window=a.restart_window, worker_health_base=a.worker_health_base,
                      worker_health_grace=a.worker_health_grace)
    return asyncio.run(pool.run_until_signalled())
