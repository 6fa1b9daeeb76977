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

    python -m tritondl.soak --jobs 5000 --torrent-jobs 100 --fail-every 50 --sample-every 500 \\
        [--file-kb 10240] [--out soak.jsonl]

Each sample is one JSON line, and a final summary follows.  The summary
gives the drift of every series after warm-up: the last sample against the
first sample taken after ``warmup`` jobs.
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

from .amqp.codec import Properties
from .amqp.connection import Connection
from .bench_job import Backend, JobStack
from .models import Download, Media, SourceType
from .utils import rawhttp


def sample(svc) -> dict:
    """One resource sample of this process."""
    import psutil
    p = psutil.Process()
    relay = rawhttp.relay_module()
    pool = relay.pool_threads() if relay is not None and hasattr(relay, "pool_threads") else None
    return {"jobs": svc.jobs_finished, "t": round(time.monotonic(), 3), "rss_mb": round(p.memory_info().rss / 2**20, 1),
            "fds": len(os.listdir("/proc/self/fd")), "os_threads": len(os.listdir("/proc/self/task")),
            "py_threads": threading.active_count(), "tasks": len(asyncio.all_tasks()),
            "pool_threads": pool, "pumps": rawhttp.active_pumps()}


def drift(samples: list[dict], warmup: int) -> dict:
    """Change of every series from the first post-warm-up sample to the last."""
    after = [s for s in samples if s["jobs"] >= warmup]
    if len(after) < 2:
        return {}
    a, b = after[0], after[-1]
    out = {}
    for k in ("rss_mb", "fds", "os_threads", "py_threads", "tasks", "pool_threads"):
        if a.get(k) is None or b.get(k) is None:
            continue
        out[k] = {"from": a[k], "to": b[k], "max": max(s[k] for s in after)}
    out["rss_drift_pct"] = round(100 * (b["rss_mb"] - a["rss_mb"]) / max(a["rss_mb"], 1e-9), 2)
    return out


async def run_soak(jobs: int, torrent_jobs: int = 0, fail_every: int = 0, sample_every: int = 500,
                   file_size: int = 10 << 20, torrent_mb: int = 8, max_retries: int = 2, warmup: int = 0,
                   on_sample=None, workdir: str | None = None) -> dict:
    st = JobStack(file_size=file_size, tag="soak", workdir=workdir)
    seed = None
    conn = None
    try:
        ends = await st.start_backends(broker=True)
        await st.setup(ends, producer=False)
        svc = st.svc
        assert svc is not None and st.cfg is not None
        st.cfg.max_retries = max_retries
        magnet = ""
        if torrent_jobs:
            from .fakes.swarm import make_payload
            src = os.path.join(st.workdir or "/tmp", "seed", "Show.S01")
            make_payload(src, {"season 1/e1.mkv": (torrent_mb << 20) // 2, "season 1/e2.mkv": (torrent_mb << 20) // 2,
                               "info.nfo": 100})
            seed = await Backend("seed", ["--path", src, "--piece-kb", "256"]).start()
            magnet = f"magnet:?xt=urn:btih:{seed.info['infohash']}&dn=Show.S01&x.pe={seed.info['endpoint']}"
        conn = await Connection.open(ends["broker"], heartbeat=0)
        ch = await conn.channel()
        await ch.confirm_select()
        origin = ends["origin"]
        # job kinds, interleaved evenly
        kinds: list[str] = []
        tor_every = max(1, jobs // torrent_jobs) if torrent_jobs else 0
        for i in range(jobs):
            if fail_every and i % fail_every == fail_every - 1:
                kinds.append("fail")
            elif tor_every and i % tor_every == tor_every // 2 and kinds.count("torrent") < torrent_jobs:
                kinds.append("torrent")
            else:
                kinds.append("http")
        n_fail = kinds.count("fail")
        expect = jobs + n_fail * max_retries        # every failing job is attempted 1 + max_retries times
        samples: list[dict] = []
        base = svc.jobs_finished
        next_sample = base
        t0 = time.monotonic()
        window = 8                                  # jobs in flight in the broker ahead of the worker

        async def publish(i: int) -> None:
            k = kinds[i]
            mid = f"soak-{i}"
            if k == "torrent":
                uri, src = magnet, SourceType.TORRENT
            elif k == "fail":
                uri, src = f"{origin}/missing/{i}.mkv", SourceType.HTTP
            else:
                uri, src = f"{origin}/synthetic/{file_size}/movie-{i}.mkv", SourceType.HTTP
            body = Download(created_at="now", media=Media(id=mid, name=mid, source=src, source_uri=uri)).encode()
            await ch.basic_publish("v1.download", f"v1.download-{i % 2}", body,
                                   Properties(delivery_mode=2, content_type="application/octet-stream"))

        sent = 0
        while svc.jobs_finished - base < expect:
            while sent < jobs and sent - (svc.jobs_finished - base) < window:
                await publish(sent)
                sent += 1
            await svc.wait_finished(svc.jobs_finished + 1, timeout=120)
            if svc.jobs_finished >= next_sample:
                gc.collect()
                s = sample(svc)
                s["jobs"] = svc.jobs_finished - base
                samples.append(s)
                if on_sample is not None:
                    on_sample(s)
                next_sample += sample_every
        dt = time.monotonic() - t0
        res = svc.results
        ok = sum(1 for r in res[-min(len(res), expect):] if r.ok)
        await asyncio.sleep(0.2)
        s = sample(svc)
        s["jobs"] = svc.jobs_finished - base
        samples.append(s)
        if on_sample is not None:
            on_sample(s)
        return {"jobs": jobs, "torrent_jobs": kinds.count("torrent"), "failing_jobs": n_fail,
                "attempts": svc.jobs_finished - base, "ok_attempts": ok, "seconds": round(dt, 2),
                "jobs_per_sec": round(jobs / dt, 1), "samples": samples, "drift": drift(samples, warmup)}
    finally:
        if conn is not None:
            await conn.close()
        if seed is not None:
            await seed.stop()
        await st.teardown()


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
    a = ap.parse_args()
    if a.cpus:
        from .parallel import topology
        if a.cpus == "auto":
            doms = topology.l3_domains()
            os.environ["TRITONDL_BENCH_FAKE_CPUS"] = ",".join(map(str, doms[1 % len(doms)]))
        topology.pin(a.cpus)
    from .utils.log import log
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
                                   a.torrent_mb, warmup=a.warmup, on_sample=emit))
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
