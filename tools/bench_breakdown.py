#!/usr/bin/env python3
"""Where does a job's time go?  Runs each stage of the flagship job in
isolation against the same out-of-process fakes ``bench.py`` uses, then the
full job, and prints one JSON line per case:

* ``fetch``   — HTTP download of the file into a job dir (no upload)
* ``upload``  — S3 PUT of a file already on disk (aws-chunked SigV4 by default)
* ``sign``    — the aws-chunked encoder alone over an in-memory buffer
* ``job``     — the whole job (consume → fetch ‖ upload → publish → ack),
                with the per-stage span medians the service records

Usage: python tools/bench_breakdown.py [--file-mb 10] [--reps 20] [--payload streaming|unsigned]
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import shutil
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tritondl.bench_job import AK, SK, Backend, JobStack  # noqa: E402
from tritondl.fetch.http import HTTPDownloader  # noqa: E402
from tritondl.fetch.registry import ProgressSink  # noqa: E402
from tritondl.ops import hashing  # noqa: E402
from tritondl.s3 import sigv4  # noqa: E402
from tritondl.s3.client import S3Client  # noqa: E402
from tritondl.s3.credentials import Static  # noqa: E402
from tritondl.utils.log import log  # noqa: E402


def _stats(xs: list[float], size: int) -> dict:
    xs = sorted(xs)
    med = statistics.median(xs)
    return {"ms_p50": round(med * 1e3, 3), "ms_min": round(xs[0] * 1e3, 3),
            "MB_per_sec_p50": round(size / med / 1e6, 1)}


async def _fetch(origin: str, size: int, reps: int, work: str) -> dict:
    dl = HTTPDownloader(progress_interval=0)
    sink = ProgressSink()
    ts = []
    try:
        for i in range(reps + 2):
            d = os.path.join(work, f"f{i}")
            os.makedirs(d)
            t = time.perf_counter()
            await dl.download(d, sink, f"{origin}/synthetic/{size}/movie-{i}.mkv")
            ts.append(time.perf_counter() - t)
            shutil.rmtree(d)
    finally:
        await dl.close()
    return _stats(ts[2:], size)


async def _upload(s3_url: str, size: int, reps: int, work: str, mode: str) -> dict:
    p = os.path.join(work, "src.mkv")
    with open(p, "wb") as f:
        f.write(os.urandom(size))
    c = S3Client(s3_url, Static(AK, SK), payload_mode=mode)
    ts = []
    try:
        if not await c.bucket_exists("bd"):
            await c.make_bucket("bd")
        for i in range(reps + 2):
            t = time.perf_counter()
            await c.put_object("bd", f"k{i}", p)
            ts.append(time.perf_counter() - t)
    finally:
        await c.close()
    return _stats(ts[2:], size)


def _sign(size: int, reps: int) -> dict:
    data = os.urandom(size)
    key = b"k" * 32
    ts = []
    for _ in range(reps + 2):
        t = time.perf_counter()
        hashing.aws_chunk_encode(key, "20260101T000000Z", "20260101/us-east-1/s3/aws4_request", "0" * 64,
                                 data, sigv4.STREAM_CHUNK, True, 0)
        ts.append(time.perf_counter() - t)
    return _stats(ts[2:], size)


async def _job(size: int, reps: int) -> dict:
    st = JobStack(file_size=size)
    await st.setup()
    try:
        await st.run_jobs(3)
        dt = await st.run_jobs(reps)
        res = st.svc.results[-reps:]  # type: ignore[union-attr]
        spans: dict[str, list[float]] = {}
        for r in res:
            for k, v in r.marks.items():
                spans.setdefault(k, []).append(v)
    finally:
        await st.teardown()
    return {"ms_per_job": round(dt / reps * 1e3, 3),
            "spans_ms_p50": {k: round(statistics.median(v) * 1e3, 3) for k, v in spans.items()}}


async def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--file-mb", type=float, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--payload", default="streaming", choices=["streaming", "unsigned", "signed"])
    a = ap.parse_args()
    log.configure("error", "")
    size = int(a.file_mb * (1 << 20))
    work = tempfile.mkdtemp(prefix="tritondl-bd-")
    og = await Backend("origin").start()
    s3 = await Backend("s3", ["--s3-store", "discard", "--access-key", AK, "--secret-key", SK]).start()
    try:
        out = {"file_bytes": size}
        out["sign"] = await asyncio.get_running_loop().run_in_executor(None, _sign, size, a.reps)
        out["fetch"] = await _fetch(og.info["url"], size, a.reps, work)
        out[f"upload_{a.payload}"] = await _upload(s3.info["url"], size, a.reps, work, a.payload)
    finally:
        await og.stop()
        await s3.stop()
        shutil.rmtree(work, ignore_errors=True)
    out["job"] = await _job(size, a.reps)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    asyncio.run(main())
