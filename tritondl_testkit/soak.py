"""Resource-leak soak of one long-running worker.

The reference's job loop runs for the life of the process
(``cmd/downloader/downloader.go:103-155``).  This worker keeps more state
across jobs than the reference did:

* pooled native buffers (relay pumps, btwire pieces) and the parked native
  task pool;
* TLS session caches and idle keep-alive connections;
* a warm DHT node;
* per-delay retry queues on the broker.

Anything that grows per job would eventually take a worker down.  The soak
runs one in-process worker (``Service``) against out-of-process fakes
(broker, origin, S3, a BitTorrent seeder).  It mixes three kinds of job:

* headline HTTP jobs;
* magnet jobs, served by the seeder (``x.pe``);
* failing jobs: a URL the origin answers with 404.  Each one is retried
  ``max_retries`` times through the broker's delay queues, then dead-lettered.

Every ``sample_every`` finished jobs it records:

* the process's RSS;
* open file descriptors;
* OS threads;
* Python threads;
* asyncio tasks;
* the native task pool's size;
* the relay's active pumps.

    python -m tritondl_testkit.soak --jobs 5000 --torrent-jobs 100 --fail-every 50 --sample-every 500 \\
        [--file-kb 10240] [--out soak.jsonl]

A job-count soak finishes in seconds, so nothing timer-driven cycles in it.
The time-based form runs for wall-clock minutes at a paced job rate:

    python -m tritondl_testkit.soak --minutes 60 --rate 50 --file-kb 1024 --torrent-every 200 \\
        --fail-every 100 --retry-delay 2 --heartbeat 10 --tls --dht-nodes 8 --out soak.jsonl

so the worker's timers go round many times: AMQP heartbeats both ways (the
fake broker sends them and drops a silent peer, as RabbitMQ does), the
delay queues' TTLs (every failing job waits ``--retry-delay`` s in one per
retry), TLS session reuse against https origin and S3, the DHT node's
token-secret rotation (5 min) and bucket refresh (15 min) against a small
local DHT of ``--dht-nodes`` nodes, and the metrics histograms.  Samples are
taken every ``--sample-seconds`` (60) and add the DHT routing-table size and
stored peers, cached TLS sessions and the number of metrics series.

Each sample is one JSON line, and a final summary follows.  The summary
gives the drift of every series after warm-up: the last sample against the
first sample taken after ``warmup`` jobs (``--warmup-minutes`` in the time
form).
"""

from __future__ import annotations

import argparse
import asyncio
import gc
import json
import os
import sys
import threading
import time

from tritondl.amqp.codec import Properties
from tritondl.amqp.connection import Connection
from .bench_job import Backend, JobStack
from tritondl.models import Download, Media, SourceType
from tritondl.utils import rawhttp


def _torrent_impl(svc):
    for impl in getattr(svc.dispatcher, "impls", []) or []:
        if hasattr(impl, "_dht"):
            return impl
    return None


def _mallinfo() -> tuple[float, float] | None:
    """glibc heap: (bytes in use, bytes the arenas hold), MiB — tells a leak
    (in-use grows) from allocator fragmentation (only the arenas grow)."""
    import ctypes

    class MI2(ctypes.Structure):
        _fields_ = [(n, ctypes.c_size_t) for n in ("arena", "ordblks", "smblks", "hblks", "hblkhd", "usmblks",
                                                    "fsmblks", "uordblks", "fordblks", "keepcost")]
    try:
        libc = ctypes.CDLL("libc.so.6")
        f = libc.mallinfo2
    except (OSError, AttributeError):
        return None
    f.restype = MI2
    m = f()
    return round((m.uordblks + m.hblkhd) / 2**20, 1), round((m.arena + m.hblkhd) / 2**20, 1)


def sample(svc) -> dict:
    """One resource sample of this process."""
    import psutil
    p = psutil.Process()
    relay = rawhttp.relay_module()
    pool = relay.pool_threads() if relay is not None and hasattr(relay, "pool_threads") else None
    out = {"jobs": svc.jobs_finished, "t": round(time.monotonic(), 3), "rss_mb": round(p.memory_info().rss / 2**20, 1),
           "fds": len(os.listdir("/proc/self/fd")), "os_threads": len(os.listdir("/proc/self/task")),
           "py_threads": threading.active_count(), "tasks": len(asyncio.all_tasks()),
           "pool_threads": pool, "pumps": rawhttp.active_pumps()}
    m = svc.metrics
    out["metrics_series"] = len(m.counters) + len(m.gauges) + len(m.hists)
    out["py_objects"] = len(gc.get_objects())
    heap = _mallinfo()
    if heap is not None:
        out["heap_in_use_mb"], out["heap_arenas_mb"] = heap
    tls = [c.cached_sessions for c in rawhttp._client_tls.values() if c is not None]
    out["tls_sessions"] = sum(tls) if tls else None
    bt = _torrent_impl(svc)
    dht = getattr(bt, "_dht", None) if bt is not None else None
    if dht is not None:
        out["dht_nodes"] = sum(len(t) for t in dht.tables.values())
        out["dht_peer_keys"] = len(dht.peers)
    return out


SERIES = ("rss_mb", "fds", "os_threads", "py_threads", "tasks", "pool_threads", "metrics_series", "tls_sessions",
          "dht_nodes", "dht_peer_keys", "py_objects", "heap_in_use_mb", "heap_arenas_mb")


def drift(samples: list[dict], warmup: int, key: str = "jobs") -> dict:
    """Change of every series from the first post-warm-up sample to the last
    (``key``: "jobs", or "minute" for time-based soaks)."""
    after = [s for s in samples if s.get(key, 0) >= warmup]
    if len(after) < 2:
        return {}
    a, b = after[0], after[-1]
    out = {}
    for k in SERIES:
        if a.get(k) is None or b.get(k) is None:
            continue
        out[k] = {"from": a[k], "to": b[k], "max": max(s[k] for s in after if s.get(k) is not None)}
    out["rss_drift_pct"] = round(100 * (b["rss_mb"] - a["rss_mb"]) / max(a["rss_mb"], 1e-9), 2)
    # the same from the medians of the first and last `w` post-warm-up samples: a
    # single sample can land on a job in flight (a torrent's pieces, a retry burst)
    w = max(1, min(5, len(after) // 4))
    med = lambda xs: sorted(xs)[len(xs) // 2]                   # noqa: E731
    m0, m1 = med([s["rss_mb"] for s in after[:w]]), med([s["rss_mb"] for s in after[-w:]])
    out["rss_median_window"] = {"samples": w, "from": m0, "to": m1,
                                "drift_pct": round(100 * (m1 - m0) / max(m0, 1e-9), 2)}
    return out


async def _local_dht(n: int) -> list:
    """``n`` DHT nodes on 127.0.0.1 that know each other: the worker's node
    bootstraps off them, so its table fills and its maintenance has peers."""
    from tritondl.fetch.bt.dht import DHTNode
    nodes = []
    for _ in range(n):
        boot = [("127.0.0.1", x.port) for x in nodes[-3:]]
        nodes.append(await DHTNode(host="127.0.0.1", bootstrap=boot, timeout=1.0).start(maintain=True))
    for x in nodes:
        await x.bootstrap()
    return nodes


async def run_soak(jobs: int, torrent_jobs: int = 0, fail_every: int = 0, sample_every: int = 500,
                   file_size: int = 10 << 20, torrent_mb: int = 8, max_retries: int = 2, warmup: int = 0,
                   on_sample=None, workdir: str | None = None, *, minutes: float = 0.0, rate: float = 0.0,
                   sample_seconds: float = 60.0, tls: bool = False, heartbeat: int = 0, retry_delay: float = 0.0,
                   torrent_every: int = 0, dht_nodes: int = 0, malloc_trim_s: float | None = None,
                   tracemalloc_frames: int = 0, concurrency: int = 1, lease_after_s: float | None = None,
                   h2_origin: bool = False, lease_s: float | None = None, stream_mbps: float = 0.0) -> dict:
    """Job-count soak (``jobs``) or, with ``minutes``, a wall-clock soak at
    ``rate`` jobs/s (0: as fast as the worker goes).  ``tracemalloc_frames``
    > 0 traces Python allocations: the summary then lists the call sites
    whose live memory grew most from the first post-warm-up sample to the
    end (``tracemalloc_growth``).  ``concurrency`` 0 is the worker's
    adaptive default; ``lease_after_s`` leases every job running longer
    (the summary then carries the lease events: taken, renewed, released,
    lost), ``lease_s`` is the lease TTL (renewed every half of it), and
    ``stream_mbps`` caps each origin / S3 stream (Mbit/s), so jobs run long
    enough for their leases to be renewed."""
    prev_mbps = os.environ.get("TRITONDL_FAKE_STREAM_MBPS")
    if stream_mbps > 0:
        os.environ["TRITONDL_FAKE_STREAM_MBPS"] = str(stream_mbps)   # the fake processes inherit it
    import tracemalloc
    timed = minutes > 0
    base_snap = None
    if tracemalloc_frames > 0:
        tracemalloc.start(tracemalloc_frames)
    st = JobStack(file_size=file_size, tag="soak", workdir=workdir, tls=tls, heartbeat=heartbeat,
                  content_check=True, concurrency=concurrency, h2_origin=h2_origin)
    if lease_after_s is not None:
        st.overrides["lease_after_s"] = lease_after_s
    if lease_s is not None:
        st.overrides["lease_s"] = lease_s
    if malloc_trim_s is not None:
        st.overrides["malloc_trim_s"] = malloc_trim_s
    seed = None
    conn = None
    dht = []
    try:
        ends = await st.start_backends(broker=True)
        if dht_nodes:
            dht = await _local_dht(dht_nodes)
            st.overrides.update(bt_bootstrap=",".join(f"127.0.0.1:{x.port}" for x in dht), bt_dht=True,
                                bt_dht_ipv6=False)
        await st.setup(ends, producer=False)
        svc = st.svc
        assert svc is not None and st.cfg is not None
        st.cfg.max_retries = max_retries
        st.cfg.retry_delay_s = retry_delay
        st.cfg.retry_backoff = 1.0
        magnet = ""
        if torrent_jobs or torrent_every:
            from .fakes.swarm import make_payload
            src = os.path.join(st.workdir or "/tmp", "seed", "Show.S01")
            make_payload(src, {"season 1/e1.mkv": (torrent_mb << 20) // 2, "season 1/e2.mkv": (torrent_mb << 20) // 2,
                               "info.nfo": 100})
            seed = await Backend("seed", ["--path", src, "--piece-kb", "256"]).start()
            magnet = f"magnet:?xt=urn:btih:{seed.info['infohash']}&dn=Show.S01&x.pe={seed.info['endpoint']}"
        conn = await Connection.open(ends["broker"], heartbeat=heartbeat)
        ch = await conn.channel()
        await ch.confirm_select()
        origin = ends["origin"]
        tor_every = torrent_every or (max(1, jobs // torrent_jobs) if torrent_jobs else 0)
        n_tor = [0]

        def kind(i: int) -> str:
            if fail_every and i % fail_every == fail_every - 1:
                return "fail"
            if tor_every and i % tor_every == tor_every // 2 and (timed or n_tor[0] < torrent_jobs):
                n_tor[0] += 1
                return "torrent"
            return "http"
        kinds: list[str] = []
        samples: list[dict] = []
        base = svc.jobs_finished
        ok0 = svc.metrics.get("jobs", status="ok")
        next_sample = base
        t0 = time.monotonic()
        next_t = t0
        end_t = t0 + minutes * 60 if timed else float("inf")
        window = 8                                  # jobs in flight in the broker ahead of the worker

        async def publish(i: int) -> None:
            k = kind(i)
            kinds.append(k)
            mid = f"soak-{i}"
            if k == "torrent":
                uri, src = magnet, SourceType.TORRENT
            elif k == "fail":
                uri, src = f"{origin}/missing/{i}.mkv", SourceType.HTTP
            else:
                uri, src = f"{origin}/synthetic/{file_size}/{st.job_name(i)}", SourceType.HTTP
            body = Download(created_at="now", media=Media(id=mid, name=mid, source=src, source_uri=uri)).encode()
            await ch.basic_publish("v1.download", f"v1.download-{i % 2}", body,
                                   Properties(delivery_mode=2, content_type="application/octet-stream"))

        def take_sample(extra: dict | None = None) -> None:
            nonlocal base_snap
            gc.collect()
            s = sample(svc)
            s.update(extra or {})
            s["jobs"] = svc.jobs_finished - base
            s["minute"] = round((time.monotonic() - t0) / 60, 2)
            if tracemalloc.is_tracing():
                s["traced_mb"] = round(tracemalloc.get_traced_memory()[0] / 2**20, 2)
                if base_snap is None and s["minute" if timed else "jobs"] >= warmup:
                    base_snap = tracemalloc.take_snapshot()
            samples.append(s)
            if on_sample is not None:
                on_sample(s)

        def expected() -> int:                      # every failing job is attempted 1 + max_retries times
            return len(kinds) + kinds.count("fail") * max_retries

        sent = 0
        while True:
            now = time.monotonic()
            more = (now < end_t) if timed else (sent < jobs)
            if not more and svc.jobs_finished - base >= expected():
                break
            while more and sent - (svc.jobs_finished - base) < window and (not rate or now >= next_t):
                await publish(sent)
                sent += 1
                next_t += 1.0 / rate if rate else 0.0
                now = time.monotonic()
                more = (now < end_t) if timed else (sent < jobs)
            wait = 1.0 if not more else max(0.0, min(1.0, next_t - time.monotonic())) if rate else None
            try:
                await svc.wait_finished(svc.jobs_finished + 1, timeout=wait if wait else 120)
            except TimeoutError:
                if not timed and not rate:
                    raise
            if timed:
                if time.monotonic() - t0 >= len(samples) * sample_seconds:
                    ok_h, why = await svc.health()          # what /healthz would answer now
                    e = svc.amqp.confirm_ewma if svc.amqp is not None else None
                    take_sample({"healthy": ok_h, **({"health_why": why[:3]} if why else {}),
                                 "confirm_ms": round(e * 1000, 3) if e is not None else None,
                                 "pipelined": svc._pipeline_now(), "concurrency_limit": svc._limit,
                                 "leases_held": len(svc.amqp._leased) if svc.amqp is not None else None})
            elif svc.jobs_finished >= next_sample:
                take_sample()
                next_sample += sample_every
        dt = time.monotonic() - t0
        n_att = svc.jobs_finished - base
        ok = int(svc.metrics.get("jobs", status="ok") - ok0)    # results[] keeps only the last 10,000
        await asyncio.sleep(0.2)
        take_sample()
        summary = {"jobs": len(kinds), "torrent_jobs": kinds.count("torrent"), "failing_jobs": kinds.count("fail"),
                   "attempts": n_att, "ok_attempts": ok, "seconds": round(dt, 2),
                   "jobs_per_sec": round(len(kinds) / dt, 1), "samples": samples,
                   "drift": drift(samples, warmup, "minute" if timed else "jobs")}
        if base_snap is not None:
            grown = tracemalloc.take_snapshot().compare_to(base_snap, "traceback")
            summary["tracemalloc_growth"] = [
                {"kb": round(g.size_diff / 1024, 1), "blocks": g.count_diff,
                 "where": [f"{fr.filename.rsplit('/', 2)[-2:]}:{fr.lineno}".replace("'", "") for fr in g.traceback][-4:]}
                for g in grown[:15]]
            tracemalloc.stop()
        summary["h2_streams"] = sum(getattr(i, "h2_streams", 0) for i in getattr(svc.dispatcher, "impls", []) or [])
        if svc.amqp is not None:
            summary["lease_stats"] = dict(svc.amqp.lease_stats)
            summary["leases_held_at_end"] = len(svc.amqp._leased)
        if timed:
            summary.update(minutes=minutes, rate=rate, tls=tls, heartbeat=heartbeat, retry_delay=retry_delay,
                           dht_nodes=dht_nodes, reconnects=svc.amqp.reconnects if svc.amqp is not None else None)
        return summary
    finally:
        if conn is not None:
            await conn.close()
        if seed is not None:
            await seed.stop()
        for x in dht:
            x.stop()
        await st.teardown()
        if stream_mbps > 0:
            if prev_mbps is None:
                os.environ.pop("TRITONDL_FAKE_STREAM_MBPS", None)
            else:
                os.environ["TRITONDL_FAKE_STREAM_MBPS"] = prev_mbps


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=5000)
    ap.add_argument("--torrent-jobs", type=int, default=100)
    ap.add_argument("--fail-every", type=int, default=50)
    ap.add_argument("--sample-every", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--file-kb", type=int, default=10240)
    ap.add_argument("--torrent-mb", type=int, default=8)
    ap.add_argument("--out", default="")
    ap.add_argument("--cpus", default="", help="pin the worker like TRITONDL_CPUS (cpulist or auto); the fakes "
                                               "go to the next L3 domain with auto")
    ap.add_argument("--minutes", type=float, default=0.0, help="wall-clock soak of this many minutes (0: --jobs)")
    ap.add_argument("--rate", type=float, default=0.0, help="jobs/s to publish (0: as fast as the worker takes them)")
    ap.add_argument("--sample-seconds", type=float, default=60.0)
    ap.add_argument("--warmup-minutes", type=float, default=5.0)
    ap.add_argument("--torrent-every", type=int, default=0, help="time form: every Nth job is a magnet job")
    ap.add_argument("--retry-delay", type=float, default=0.0, help="seconds each failing job waits in a delay queue")
    ap.add_argument("--heartbeat", type=int, default=0, help="AMQP heartbeat (s), broker and worker")
    ap.add_argument("--tls", action="store_true", help="origin and S3 over https")
    ap.add_argument("--rtt-ms", type=float, default=0.0, help="emulated round trip of the fakes (ms)")
    ap.add_argument("--dht-nodes", type=int, default=0, help="local DHT nodes the worker bootstraps from")
    ap.add_argument("--malloc-trim", type=float, default=None, help="worker's malloc_trim period (s; 0 = off)")
    ap.add_argument("--concurrency", type=int, default=1, help="jobs in flight (0: the worker's adaptive default)")
    ap.add_argument("--lease-after", type=float, default=None, help="lease every job running longer than this (s)")
    ap.add_argument("--h2-origin", action="store_true", help="with --tls: the origin serves HTTP/2")
    ap.add_argument("--lease-ttl", type=float, default=None, help="lease TTL (s), renewed every half of it")
    ap.add_argument("--stream-mbps", type=float, default=0.0,
                    help="cap each fake origin / S3 stream (Mbit/s): long jobs whose leases renew")
    ap.add_argument("--tracemalloc", type=int, default=0,
                    help="trace Python allocations with this many frames; the summary lists the biggest growth")
    a = ap.parse_args()
    if a.rtt_ms > 0:
        os.environ["TRITONDL_FAKE_RTT_MS"] = str(a.rtt_ms)   # the fake processes inherit it
    if a.cpus:
        from tritondl.parallel import topology
        if a.cpus == "auto":
            doms = topology.l3_domains()
            os.environ["TRITONDL_BENCH_FAKE_CPUS"] = ",".join(map(str, doms[1 % len(doms)]))
        topology.pin(a.cpus)
    from tritondl.utils.log import log
    log.configure("warning", "")
    fh = open(a.out, "w") if a.out else None

    def emit(s: dict) -> None:
        line = json.dumps(s)
        print(line, flush=True)
        if fh is not None:
            fh.write(line + "\n")
            fh.flush()
    try:
        res = asyncio.run(run_soak(a.jobs, a.torrent_jobs, a.fail_every, a.sample_every, a.file_kb << 10,
                                   a.torrent_mb, warmup=(a.warmup_minutes if a.minutes else a.warmup),
                                   on_sample=emit, minutes=a.minutes, rate=a.rate, sample_seconds=a.sample_seconds,
                                   tls=a.tls, heartbeat=a.heartbeat, retry_delay=a.retry_delay,
                                   torrent_every=a.torrent_every, dht_nodes=a.dht_nodes,
                                   malloc_trim_s=a.malloc_trim, tracemalloc_frames=a.tracemalloc,
                                   concurrency=a.concurrency, lease_after_s=a.lease_after,
                                   h2_origin=a.h2_origin, lease_s=a.lease_ttl, stream_mbps=a.stream_mbps))
    finally:
        if fh is not None:
            fh.close()
    summary = {k: v for k, v in res.items() if k != "samples"}
    print(json.dumps({"summary": summary}), flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps({"summary": summary}) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
