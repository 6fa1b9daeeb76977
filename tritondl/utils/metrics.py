"""Minimal Prometheus-text metrics (the reference had none):
counters, gauges and fixed-bucket histograms, plus an optional aiohttp
``/metrics`` + ``/healthz`` endpoint.  Single event loop → no locking
needed on the hot path; the exposition snapshot is taken on the loop too.
"""

from __future__ import annotations

import bisect
import inspect
import time
from dataclasses import dataclass, field

_DEF_BUCKETS = (0.01, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60, 300, 900, 3600)


@dataclass
class _Hist:
    buckets: tuple[float, ...] = _DEF_BUCKETS
    counts: list[int] = field(default_factory=list)
    total: float = 0.0
    n: int = 0

    def __post_init__(self) -> None:
        self.counts = [0] * (len(self.buckets) + 1)

    def observe(self, v: float) -> None:
        self.counts[bisect.bisect_left(self.buckets, v)] += 1
        self.total += v
        self.n += 1


class Metrics:
    def __init__(self, prefix: str = "tritondl") -> None:
        self.prefix = prefix
        self.counters: dict[tuple[str, tuple], float] = {}
        self.gauges: dict[tuple[str, tuple], float] = {}
        self.hists: dict[tuple[str, tuple], _Hist] = {}
        self.started = time.time()
        self.collectors: list = []      # callables run before each render (gauges computed on scrape)

    @staticmethod
    def _k(name: str, labels: dict | None) -> tuple[str, tuple]:
        return name, tuple(sorted((labels or {}).items()))

    def inc(self, name: str, v: float = 1.0, **labels) -> None:
        k = self._k(name, labels)
        self.counters[k] = self.counters.get(k, 0.0) + v

    def set(self, name: str, v: float, **labels) -> None:
        self.gauges[self._k(name, labels)] = v

    def observe(self, name: str, v: float, **labels) -> None:
        k = self._k(name, labels)
        h = self.hists.get(k)
        if h is None:
            h = self.hists[k] = _Hist()
        h.observe(v)

    def get(self, name: str, **labels) -> float:
        k = self._k(name, labels)
        return self.counters.get(k, self.gauges.get(k, 0.0))

    def render(self) -> str:
        """Prometheus text exposition (format 0.0.4): one ``# HELP`` / ``# TYPE``
        pair per family, then its samples; label values escaped."""
        for fn in self.collectors:
            fn()
        p = self.prefix
        out: list[str] = []

        def esc(v) -> str:
            return str(v).replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')

        def lab(items: tuple, extra: str = "") -> str:
            parts = [f'{k}="{esc(v)}"' for k, v in items]
            if extra:
                parts.append(extra)
            return "{" + ",".join(parts) + "}" if parts else ""

        def head(name: str, kind: str) -> None:
            out.append(f"# HELP {name} {HELP.get(name[len(p) + 1:], name)}")
            out.append(f"# TYPE {name} {kind}")

        last = None
        for (n, ls), v in sorted(self.counters.items()):
            if n != last:
                head(f"{p}_{n}_total", "counter")
                last = n
            out.append(f"{p}_{n}_total{lab(ls)} {v}")
        last = None
        for (n, ls), v in sorted(self.gauges.items()):
            if n != last:
                head(f"{p}_{n}", "gauge")
                last = n
            out.append(f"{p}_{n}{lab(ls)} {v}")
        last = None
        for (n, ls), h in sorted(self.hists.items(), key=lambda x: x[0]):
            if n != last:
                head(f"{p}_{n}", "histogram")
                last = n
            acc = 0
            for b, c in zip(h.buckets, h.counts):
                acc += c
                le = 'le="%s"' % b
                out.append(f"{p}_{n}_bucket{lab(ls, le)} {acc}")
            le = 'le="+Inf"'
            out.append(f"{p}_{n}_bucket{lab(ls, le)} {h.n}")
            out.append(f"{p}_{n}_sum{lab(ls)} {h.total}")
            out.append(f"{p}_{n}_count{lab(ls)} {h.n}")
        head(f"{p}_uptime_seconds", "gauge")
        out.append(f"{p}_uptime_seconds {time.time() - self.started:.3f}")
        return "\n".join(out) + "\n"


# one line per metric family (name without the prefix; counters without "_total")
HELP = {
    "jobs_total": "job attempts by status (ok, failed with its stage, busy, poison, duplicate)",
    "jobs_inflight": "jobs being processed by this worker",
    "jobs_retried_total": "failed jobs scheduled for a retry (broker delay queue or parked in-process)",
    "jobs_parked_total": "retries waited in-process because the broker refused the delay queue or DLQ",
    "jobs_parked_waiting": "deliveries waiting in-process right now (parked)",
    "jobs_poison_parked": "jobs past max_retries parked because the dead-letter topic is unreachable (never re-run)",
    "consumer_active": "1 while the shard queue has a live consumer of this worker, else 0",
    "consumers_paused": "1 while this worker's consumers are paused on purpose (a long job holds every slot: hand-back)",
    "last_job_finished_age_seconds": "seconds since this worker last recorded a job result (or started)",
    "broker_down_seconds": "seconds the broker connection has been down (0 while up)",
    "pipeline_commit_active": "1 while job commits are pipelined (the publish -> confirm round trip is long enough)",
    "jobs_dead_lettered_total": "jobs published to the dead-letter topic after max_retries",
    "jobs_handed_back_total": "buffered deliveries given back to the broker while a long job held every slot",
    "stale_job_dirs_removed_total": "job dirs removed after TRITONDL_STALE_JOB_DAYS untouched (no worker held them)",
    "jobs_dropped_total": "jobs nacked without requeue after max_retries (drop_failed)",
    "bytes_uploaded_total": "bytes uploaded to S3 by finished jobs",
    "job_seconds": "time from delivery to ack of successful jobs",
    "stage_seconds": "time per job stage (download, upload)",
    "malloc_trims_total": "malloc_trim calls that returned memory to the OS",
    "pool_workers_live": "pool: workers not given up on",
    "pool_workers_given_up": "pool: crash-looping workers given up on",
    "pool_workers_unhealthy": "pool: running workers whose own /healthz answered 503 (or not at all) at the last probe",
    "pool_worker_restarts_total": "pool: worker restarts by rank",
    "uptime_seconds": "seconds since the process's metrics started",
    "lease_returns_total": "jobs that came back because the lease of the worker running them ran out",
    "done_ledger_swept_total": "done-ledger entries removed past their TTL",
    "concurrency_limit": "jobs this worker may run at once now (adaptive concurrency, or the fixed TRITONDL_CONCURRENCY)",
    "concurrency_changes_total": "changes of the adaptive concurrency limit",
    "leases_held": "leased deliveries (job running, copy held by the broker) not settled yet",
    "lease_events": "job lease operations since start by kind (taken, renewed, released, lost, requeued, refused)",
}


async def serve_metrics(metrics: Metrics, addr: str, health=None):
    """Start ``/metrics`` and ``/healthz`` on ``host:port``; returns the runner."""
    from aiohttp import web

    host, _, port = addr.rpartition(":")
    app = web.Application()

    async def m(_req):
        return web.Response(text=metrics.render(), content_type="text/plain")

    async def hz(_req):
        """``health()`` may return a bool or (bool, [reasons]), or an awaitable of either."""
        r = True if health is None else health()
        if inspect.isawaitable(r):
            r = await r
        ok, why = (r[0], list(r[1])) if isinstance(r, tuple) else (bool(r), [])
        text = "ok" if ok else "unhealthy" + "".join(f"\n{w}" for w in why)
        return web.Response(status=200 if ok else 503, text=text + "\n")

    app.router.add_get("/metrics", m)
    app.router.add_get("/healthz", hz)
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, host or "0.0.0.0", int(port))
    await site.start()
    return runner
