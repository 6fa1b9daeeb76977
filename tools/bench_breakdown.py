#!/usr/bin/env python3
"""Where does a job's time go?  Runs each stage of the flagship job in
isolation against the same out-of-process fakes ``bench.py`` uses, then the
full job, and prints one JSON line per case:

* ``fetch``   — HTTP download of the file into a job dir (no upload)
* ``upload``  — S3 PUT of a file already on disk (aws-chunked SigV4 by default)
* ``upload_*_nullsink`` — the same PUT into a sink that ignores the body
                (the client's share of the upload)
* ``sign``    — the aws-chunked encoder alone over an in-memory buffer
* ``job``     — the whole job (consume → fetch ‖ upload → publish → ack),
                with the per-stage span medians the service records

Usage: python tools/bench_breakdown.py [--file-mb 10] [--reps 20] [--payload streaming|unsigned] [--tls]
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

from tritondl_testkit.bench_job import AK, SK, Backend, JobStack  # noqa: E402
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


def _patch_defaults(cls, kw: str, value: int) -> None:
    """Override one keyword default of ``cls.__init__`` for every instance
    this process creates (the job stack builds its own clients)."""
    if not value:
        return
    orig = cls.__init__

    def init(self, *args, **kwargs):
        kwargs.setdefault(kw, value)
        orig(self, *args, **kwargs)
    cls.__init__ = init


async def _fetch(origin: str, size: int, reps: int, work: str, ca_file: str = "") -> dict:
    dl = HTTPDownloader(progress_interval=0, ca_file=ca_file)
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


async def _upload(s3_url: str, size: int, reps: int, work: str, mode: str, make_bucket: bool = True,
                  single: bool = False, ca_file: str = "") -> dict:
    p = os.path.join(work, "src.mkv")
    with open(p, "wb") as f:
        f.write(os.urandom(size))
    c = S3Client(s3_url, Static(AK, SK), payload_mode=mode, ca_file=ca_file,
                 **({"multipart_threshold": 1 << 62} if single else {}))
    ts = []
    try:
        if make_bucket and not await c.bucket_exists("bd"):
            await c.make_bucket("bd")
        for i in range(reps + 2):
            t = time.perf_counter()
            await c.put_object("bd", f"k{i}", p)
            ts.append(time.perf_counter() - t)
    finally:
        await c.close()
    return _stats(ts[2:], size)


class _NullSink(asyncio.Protocol):
    """HTTP/1.1 sink: reads each request body by Content-Length, answers 200
    without looking at it — the client side of an upload, isolated."""

    def connection_made(self, t) -> None:
        self.t, self.buf, self.need, self.got = t, b"", None, 0

    def data_received(self, d: bytes) -> None:
        if self.need is None:
            self.buf += d
            i = self.buf.find(b"\r\n\r\n")
            if i < 0:
                return
            cl = 0
            for line in self.buf[:i].split(b"\r\n")[1:]:
                k, _, v = line.partition(b":")
                if k.strip().lower() == b"content-length":
                    cl = int(v)
            self.need, self.got, self.buf = cl, len(self.buf) - i - 4, b""
        else:
            self.got += len(d)
        if self.got >= self.need:
            self.t.write(b'HTTP/1.1 200 OK\r\nContent-Length: 0\r\nETag: "0"\r\n\r\n')
            self.need, self.got = None, 0


async def _upload_null(size: int, reps: int, work: str, mode: str) -> dict:
    srv = await asyncio.get_running_loop().create_server(_NullSink, "127.0.0.1", 0)
    try:
        port = srv.sockets[0].getsockname()[1]
        # the sink speaks no multipart XML: large files go as one PUT (single-stream client rate)
        return await _upload(f"http://127.0.0.1:{port}", size, reps, work, mode, make_bucket=False, single=True)
    finally:
        srv.close()


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


def _trace_summary() -> dict:
    """Median time of each traced data-plane event relative to its job's start."""
    from tritondl.utils import rawhttp
    tr = rawhttp.TRACE or []
    rel: dict[str, list[float]] = {}
    t0 = None
    for ev, t in tr:
        if ev == "job_start":
            t0 = t
            continue
        if t0 is not None:
            rel.setdefault(ev, []).append(t - t0)
    return {k: round(statistics.median(v) * 1e3, 3) for k, v in rel.items()}


async def _job(size: int, reps: int, tls: bool = False) -> dict:
    from tritondl.utils import rawhttp
    st = JobStack(file_size=size, tls=tls)
    await st.setup()
    try:
        await st.run_jobs(3)
        if rawhttp.TRACE is not None:
            rawhttp.TRACE.clear()
        dt = await st.run_jobs(reps)
        res = st.svc.results[-reps:]  # type: ignore[union-attr]
        spans: dict[str, list[float]] = {}
        for r in res:
            for k, v in r.marks.items():
                spans.setdefault(k, []).append(v)
    finally:
        await st.teardown()
    return {"ms_per_job": round(dt / reps * 1e3, 3),
            "spans_ms_p50": {k: round(statistics.median(v) * 1e3, 3) for k, v in spans.items()},
            "trace_ms_p50": _trace_summary()}


async def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--file-mb", type=float, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--payload", default="streaming", choices=["streaming", "unsigned", "signed"])
    ap.add_argument("--http-bufsize", type=int, default=0, help="worker HTTP client read_bufsize (0 = default)")
    ap.add_argument("--s3-bufsize", type=int, default=0, help="fake S3 server read_bufsize (0 = default)")
    ap.add_argument("--io-block", type=int, default=0, help="S3 upload read/sign block (0 = default)")
    ap.add_argument("--tls", action="store_true", help="origin and S3 over https (native TLS data plane)")
    ap.add_argument("--cpus", default="auto", choices=["auto", "none"],
                    help="auto: this process on one L3 domain and the fakes on the next, as bench.py")
    a = ap.parse_args()
    if a.cpus == "auto":
        from tritondl.parallel import topology
        doms = topology.l3_domains()
        os.environ["TRITONDL_BENCH_FAKE_CPUS"] = ",".join(map(str, doms[1 % len(doms)]))
        os.sched_setaffinity(0, doms[0])
    if a.s3_bufsize:
        os.environ["TRITONDL_FAKE_S3_READ_BUFSIZE"] = str(a.s3_bufsize)
    _patch_defaults(HTTPDownloader, "read_bufsize", a.http_bufsize)
    _patch_defaults(S3Client, "io_block", a.io_block)
    log.configure("error", "")
    size = int(a.file_mb * (1 << 20))
    work = tempfile.mkdtemp(prefix="tritondl-bd-")
    stack = JobStack(file_size=size, tls=a.tls, workdir=os.path.join(work, "stack"))
    os.makedirs(stack.workdir)
    eps = await stack.start_backends(broker=False)
    ca = eps.get("ca_file", "")
    payload = a.payload if not a.tls or a.payload != "streaming" else "unsigned"   # minio-go's https choice
    try:
        out = {"file_bytes": size, "tls": a.tls}
        out["sign"] = await asyncio.get_running_loop().run_in_executor(None, _sign, size, a.reps)
        out["fetch"] = await _fetch(eps["origin"], size, a.reps, work, ca)
        out[f"upload_{payload}"] = await _upload(eps["s3"], size, a.reps, work, payload, ca_file=ca)
        if not a.tls:
            out[f"upload_{payload}_nullsink"] = await _upload_null(size, a.reps, work, payload)
    finally:
        for b in stack.backends:
            await b.stop()
        shutil.rmtree(work, ignore_errors=True)
    out["job"] = await _job(size, a.reps, a.tls)
    out["knobs"] = {"http_bufsize": a.http_bufsize, "s3_bufsize": a.s3_bufsize, "io_block": a.io_block}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    asyncio.run(main())
