#!/usr/bin/env python3
"""Node throughput benchmark ("8 worker processes × 100 small
HTTP jobs → jobs/sec").

The fake broker, origin and S3 run as separate processes; ``WorkerPool``
starts N real worker processes (``python -m tritondl``, competing consumers on
the sharded queues, exactly the production launcher); this process publishes
the jobs and counts the ``v1.convert`` messages.  Warm-up: one job per worker
first, so every worker has connected and consumed before the clock starts.

    python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 1024   # 800 jobs
    python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4

``--nodes K`` runs K origin and K S3 processes (CDN edges / MinIO nodes): job
URLs round-robin over the origins and worker r uploads to S3 node r % K, so a
single-process fake does not cap the node.  ONE broker either way.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


async def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--jobs", type=int, default=0, help="total jobs (default: workers x jobs-per-worker)")
    ap.add_argument("--jobs-per-worker", type=int, default=100)
    ap.add_argument("--file-kb", type=int, default=1024)
    ap.add_argument("--concurrency", type=int, default=1, help="jobs in flight per worker (reference: 1)")
    ap.add_argument("--nodes", type=int, default=1, help="origin + S3 fake processes (sharded)")
    ap.add_argument("--placement", default="l3", choices=["l3", "l3-fixed", "slice"],
                    help="worker CPU sets: one L3 domain each, the idlest of each worker's share (default), "
                         "one L3 domain each at fixed strides (the plan before load sampling), or "
                         "consecutive CPU-id slices")
    ap.add_argument("--s3-hash-device", default="cpu", choices=["cpu", "gpu"],
                    help="workers hash aws-chunked chunks on SHA-NI or the HIP kernel")
    a = ap.parse_args()
    a.jobs = a.jobs or a.workers * a.jobs_per_worker
    from tritondl.amqp.codec import Properties
    from tritondl.amqp.connection import Connection
    from tritondl_testkit.bench_job import AK, SK, Backend
    from tritondl.models import Convert, Download, Media, SourceType
    from tritondl.parallel import WorkerPool, plan

    work = tempfile.mkdtemp(prefix="tdl-poolbench-", dir=os.environ.get("TMPDIR", "/tmp"))
    backends: list[Backend] = []
    pool = None
    prod = None
    try:
        bk = await Backend("broker").start()
        backends = [bk]
        origins, s3s = [], []
        for _ in range(max(1, a.nodes)):
            og = await Backend("origin").start()
            s3 = await Backend("s3", ["--s3-store", "discard", "--access-key", AK, "--secret-key", SK]).start()
            origins.append(og.info["url"])
            s3s.append(s3.info["url"])
            backends += [og, s3]
        env = {"RABBITMQ_ENDPOINT": bk.info["endpoint"], "RABBITMQ_USERNAME": "guest",
               "RABBITMQ_PASSWORD": "guest", "AWS_ACCESS_KEY_ID": AK,
               "AWS_SECRET_ACCESS_KEY": SK, "PYTHONPATH": ROOT, "TRITONDL_RETRY_DELAY": "0",
               "TRITONDL_BT_DHT": "0", "LOG_LEVEL": "warning", "TRITONDL_PROGRESS_LOG_INTERVAL": "0",
               "TRITONDL_CLEANUP": "1", "TRITONDL_CONCURRENCY": str(a.concurrency),
               "TRITONDL_PREFETCH": str(a.concurrency), "TRITONDL_GPU_VERIFY": "off",
               "TRITONDL_S3_HASH_DEVICE": a.s3_hash_device}
        ncpu = len(os.sched_getaffinity(0))
        # --placement l3: one CCD per worker (topology.plan); slice: consecutive CPU ids
        if a.placement == "l3":
            specs = plan(a.workers, gpus=0)
        elif a.placement == "l3-fixed":
            from tritondl.parallel.topology import l3_domains
            specs = plan(a.workers, gpus=0, busy=[0.0] * len(l3_domains()))
        else:
            specs = plan(a.workers, gpus=0, cpus=ncpu, cpus_per_worker=max(1, ncpu // a.workers))
        pool = WorkerPool(specs,
                          env=env, cwd=work, grace=10,
                          worker_env=lambda r: {"S3_ENDPOINT": s3s[r % len(s3s)]})
        await pool.start()
        prod = await Connection.open(bk.info["url"], heartbeat=0)
        pch = await prod.channel()
        await pch.confirm_select()
        cch = await prod.channel()
        done: list[float] = []
        ids: set[str] = set()
        got = asyncio.Event()
        target = [0]

        def on_convert(m) -> None:
            c = Convert.decode(m.body)
            if c.media is not None and c.media.id not in ids:
                ids.add(c.media.id)
                done.append(time.perf_counter())
                if len(done) >= target[0]:
                    got.set()
            asyncio.ensure_future(m.ack())
        await pch.exchange_declare("v1.download", "direct", durable=True)
        for i in range(2):
            await pch.queue_declare(f"v1.download-{i}", durable=True)
            await pch.queue_bind(f"v1.download-{i}", "v1.download", f"v1.download-{i}")
            await cch.queue_declare(f"v1.convert-{i}", durable=True)
            await cch.basic_consume(f"v1.convert-{i}", on_convert)
        size = a.file_kb << 10
        n_sub = [0]

        async def submit(n: int) -> None:
            for _ in range(n):
                i = n_sub[0]
                n_sub[0] += 1
                url = f"{origins[i % len(origins)]}/synthetic/{size}/clip-{i}.mkv"
                body = Download(created_at="now", media=Media(id=f"pool-{i}", name=f"clip {i}",
                                                              source=SourceType.HTTP, source_uri=url)).encode()
                await pch.basic_publish("v1.download", f"v1.download-{i % 2}", body,
                                        Properties(delivery_mode=2, content_type="application/octet-stream"))

        # warm-up: every worker connected and through one job
        target[0] = 2 * a.workers
        await submit(target[0])
        await asyncio.wait_for(got.wait(), 180)
        got.clear()
        base = len(done)
        target[0] = base + a.jobs
        t0 = time.perf_counter()
        await submit(a.jobs)
        await asyncio.wait_for(got.wait(), 600)
        dt = time.perf_counter() - t0
        print(json.dumps({"metric": "pool_jobs_per_sec", "value": round(a.jobs / dt, 2), "seconds": round(dt, 3),
                          "workers": a.workers, "placement": a.placement, "jobs": a.jobs, "file_kb": a.file_kb,
                          "concurrency_per_worker": a.concurrency, "fake_nodes": a.nodes,
                          "ingest_MB_per_sec": round(a.jobs * size / dt / 1e6, 1)}), flush=True)
    finally:
        if prod is not None:
            await prod.close()
        if pool is not None:
            await pool.stop()
        for b in backends:
            await b.stop()
        shutil.rmtree(work, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(asyncio.run(main()))
