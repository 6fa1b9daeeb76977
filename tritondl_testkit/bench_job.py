"""End-to-end job harness: the BASELINE.json config "Single HTTP download
job via local RabbitMQ, 10 MB file", used by ``bench.py``, ``smoke()`` and
the integration tests.

Layout: the fake broker, HTTP origin and S3 each run in their OWN process
(``tritondl_testkit.fakes.serve``) — as the real RabbitMQ / media server / MinIO
would — and the worker (``Service``) runs in this process exactly as in
production (multi-rank: one shared broker, per-rank origin + S3 nodes, see
:class:`JobStack`): AMQP consume from ``v1.download-{0,1}`` → HTTP
fetch into ``downloading/<id>/`` → select → SigV4 aws-chunked PUT to
``triton-staging/<id>/original/<b64>`` → publish ``v1.convert`` → ack.
A producer connection publishes the ``api.Download`` jobs; completion is
observed as the job's ack, and each ``Convert`` is checked on the way out.

Every job fetches a payload of its own (variant ``i % R`` of the synthetic
file, ``R`` larger than the spare-file pool, :mod:`tritondl_testkit.fakes.payload`)
and the S3 fake refuses any PUT whose 64 KiB-leaf SHA-256 list is not that
variant's: a worker that uploads stale or torn bytes fails the run.
"""

from __future__ import annotations

import asyncio
import contextlib
import hashlib
import json
import os
import shutil
import sys
import tempfile
import time
from dataclasses import dataclass, field

from tritondl.amqp.client import Client
from tritondl.amqp.codec import Properties
from tritondl.amqp.connection import Connection
from tritondl.models import Convert, Download, Media, SourceType
from tritondl.s3.client import S3Client
from tritondl.s3.credentials import Static
from tritondl.s3.uploader import Uploader
from tritondl.service import Service
from tritondl.utils.config import Config

AK, SK = "benchaccess", "benchsecret"


class Backend:
    def __init__(self, kind: str, extra: list[str] | None = None, module: str = "tritondl_testkit.fakes.serve") -> None:
        self.kind = kind
        self.extra = extra or []
        self.module = module
        self.proc: asyncio.subprocess.Process | None = None
        self.info: dict = {}

    async def start(self) -> "Backend":
        args = [self.kind] if self.module == "tritondl_testkit.fakes.serve" else []
        # (TRITONDL_BENCH_FAKE_CPUS, if set, is inherited: the child pins itself first
        # thing, topology.pin_from_env — no preexec_fn in a process that has threads)
        self.proc = await asyncio.create_subprocess_exec(
            sys.executable, "-m", self.module, *args, *self.extra,
            stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
            cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert self.proc.stdout is not None
        line = await asyncio.wait_for(self.proc.stdout.readline(), 120)
        if not line:
            raise RuntimeError(f"fake {self.kind} failed to start")
        self.info = json.loads(line)
        return self

    async def request(self, msg: dict, timeout: float = 900) -> dict:
        """One JSON command on stdin, one JSON reply on stdout (the producer)."""
        assert self.proc is not None and self.proc.stdin is not None and self.proc.stdout is not None
        self.proc.stdin.write((json.dumps(msg) + "\n").encode())
        await self.proc.stdin.drain()
        line = await asyncio.wait_for(self.proc.stdout.readline(), timeout)
        if not line:
            raise RuntimeError(f"{self.kind} process exited")
        out = json.loads(line)
        if "error" in out:
            raise RuntimeError(f"{self.kind}: {out['error']}")
        return out

    async def stop(self) -> None:
        p = self.proc
        if p is None:
            return
        with contextlib.suppress(Exception):
            if p.stdin:
                p.stdin.close()
        try:
            await asyncio.wait_for(p.wait(), 10)
        except asyncio.TimeoutError:
            p.kill()  # our own child, by PID
            await p.wait()
        self.proc = None


@dataclass
class JobStack:
    """Fakes + worker + producer for N synthetic jobs.

    Single-worker mode (``setup()``): this stack starts its own broker,
    origin and S3.  Shared mode (multi-rank bench): rank 0 starts the ONE
    broker every worker competes on (``start_backends(broker=True)``), each
    rank starts its own origin and S3 node (sharded, like CDN edges / MinIO
    nodes — a single-process fake would cap the node), the endpoints are
    exchanged, and ``setup(endpoints, origins, producer=rank == 0)`` wires the
    worker to them; only rank 0 publishes jobs and counts ``v1.convert``."""

    file_size: int = 10 * 1024 * 1024
    concurrency: int = 1
    prefetch: int = 1
    workdir: str | None = None
    inproc: bool = False
    tag: str = "r0"
    http_probe_bytes: int = -1       # -1: worker default (Config)
    http_segments: int = 0           # 0: worker default
    http_stripe_bytes: int = -1      # -1: worker default
    s3_part_size: int = 0            # 0: worker default
    s3_multipart_threshold: int = 0  # 0: worker default
    sign_threads: int = 0            # 0: worker default
    tls: bool = False                # origin + S3 over https (OpenSSL in the native data plane)
    h2_origin: bool = False          # with tls: the origin serves HTTP/2 (ALPN h2) instead of HTTP/1.1
    payload_mode: str = ""           # "" → aws-chunked over http, unsigned over https (minio-go's choice)
    hash_device: str = "cpu"         # aws-chunked chunk SHA-256s: cpu (SHA-NI) | gpu (HIP)
    cleanup: bool = True             # delete (or recycle) each job's dir once settled; False = the reference (B15)
    recycle_bytes: int = -1          # -1: worker default (Config); 0: delete every file
    variants: int = -1               # payload variants; -1: more than the spare pool can hold, 0: one payload
    content_check: bool = True       # S3 refuses PUTs whose content is not the origin's variant
    heartbeat: int = 0               # AMQP heartbeat (s) the broker proposes and the worker uses (0: off)
    overrides: dict = field(default_factory=dict)    # worker Config fields set before the service starts
    cfg: Config | None = None
    backends: list = field(default_factory=list)
    svc: Service | None = None
    producer: Connection | None = None               # in-process producer (inproc stacks: smoke, tests)
    producer_proc: Backend | None = None             # the producer / convert counter process (benches)
    broker_pid: int = 0
    last_run: dict = field(default_factory=dict)     # the producer's report of the last run
    origin_urls: list = field(default_factory=list)
    _n: int = 0

    def resolved_recycle_bytes(self) -> int:
        if self.recycle_bytes >= 0:
            return self.recycle_bytes
        return int(os.environ.get("TRITONDL_RECYCLE_BYTES", Config().recycle_bytes))

    def resolved_variants(self) -> int:
        """More variants than spare files the pool can hold (max 64 files,
        service.py), so a recycled spare never holds the new job's own bytes."""
        if self.variants >= 0:
            return self.variants
        depth = min(64, self.resolved_recycle_bytes() // max(1, self.file_size)) if self.cleanup else 0
        return depth + 3

    def _variant_args(self) -> list[str]:
        r = self.resolved_variants()
        return ["--variants", str(r), "--variant-size", str(self.file_size)] if r else []

    def _tls_files(self) -> tuple[str, str, str]:
        """(ca_file, cert_file, key_file) of a throwaway PKI in the workdir."""
        from tritondl.utils import rawhttp
        assert self.workdir is not None
        ca, cert, key = rawhttp.relay_module().make_test_pki(["127.0.0.1", "localhost"])
        paths = []
        for name, pem in (("ca.pem", ca), ("cert.pem", cert), ("key.pem", key)):
            pth = os.path.join(self.workdir, name)
            with open(pth, "w") as f:
                f.write(pem)
            paths.append(pth)
        return paths[0], paths[1], paths[2]

    async def start_backends(self, broker: bool = True) -> dict:
        """Start this stack's fakes; returns their URLs (``broker`` only if asked)."""
        if self.workdir is None:
            self.workdir = tempfile.mkdtemp(prefix="tritondl-bench-")
        out: dict = {}
        if self.inproc:
            from .fakes.broker import Broker
            from .fakes.s3 import FakeS3
            from .fakes.serve import SyntheticOrigin
            tls = None
            if self.tls:
                ca_file, cert_f, key_f = self._tls_files()
                with open(cert_f) as f1, open(key_f) as f2:
                    tls = (f1.read(), f2.read())
                out["ca_file"] = ca_file
            if broker:
                b = await Broker(heartbeat=self.heartbeat).start()
                self.backends.append(b)
                out["broker"] = b.url
            from .fakes.payload import Expectations
            r = self.resolved_variants()
            if self.h2_origin and tls is not None:
                from .fakes.serve import SyntheticH2Origin
                o = SyntheticH2Origin(cert_pem=tls[0], key_pem=tls[1])
            else:
                o = SyntheticOrigin(tls=tls)
            o.precompute(self.file_size, r)
            await o.start()
            expect = Expectations(self.file_size, r) if r and self.content_check else None
            s3 = await FakeS3(store="memory", access_key=AK, secret_key=SK, tls=tls, expect=expect).start()
            self.backends += [o, s3]
            out["origin"] = f"{'https' if tls else 'http'}://{o.host}:{o.port}"
            out["s3"] = s3.endpoint
            return out
        tls_args: list[str] = []
        if self.tls:
            ca_file, cert_f, key_f = self._tls_files()
            tls_args = ["--tls-cert", cert_f, "--tls-key", key_f]
            out["ca_file"] = ca_file
        if broker:
            bk = await Backend("broker", ["--heartbeat", str(self.heartbeat)] if self.heartbeat else []).start()
            self.backends.append(bk)
            out["broker"] = bk.info["url"]
            self.broker_pid = bk.proc.pid if bk.proc is not None else 0
        va = self._variant_args()
        og = await Backend("h2origin" if self.h2_origin and self.tls else "origin", [*tls_args, *va]).start()
        s3 = await Backend("s3", ["--s3-store", "discard", "--access-key", AK, "--secret-key", SK, *tls_args,
                                  *(va if self.content_check else [])]).start()
        self.backends += [og, s3]
        out["origin"], out["s3"] = og.info["url"], s3.info["url"]
        return out

    async def setup(self, endpoints: dict | None = None, origins: list[str] | None = None,
                    producer: bool = True) -> None:
        if endpoints is None:
            endpoints = await self.start_backends(broker=True)
        if self.workdir is None:
            self.workdir = tempfile.mkdtemp(prefix="tritondl-bench-")
        broker_url, s3_url = endpoints["broker"], endpoints["s3"]
        self.origin_urls = list(origins or [endpoints["origin"]])
        cfg = Config()
        cfg.download_dir = os.path.join(self.workdir, "downloading")
        cfg.concurrency = self.concurrency
        cfg.prefetch = self.prefetch
        # cleanup keeps disk bounded across thousands of bench jobs; the reference never
        # deleted (B15): cleanup=False is its mode.  Spare-file recycling (utils/spares.py)
        # is on with cleanup; recycle_bytes 0 = the A/B switch
        cfg.cleanup = self.cleanup
        cfg.recycle_bytes = self.resolved_recycle_bytes()
        cfg.retry_delay_s = 0.0
        cfg.max_retries = 0
        cfg.progress_log_interval_s = 0
        cfg.heartbeat_s = self.heartbeat
        cfg.ca_file = endpoints.get("ca_file", "")
        for var, attr in (("TRITONDL_MALLOC_MMAP_THRESHOLD", "malloc_mmap_threshold"),
                          ("TRITONDL_MALLOC_ARENA_MAX", "malloc_arena_max"),
                          ("TRITONDL_MALLOC_TRIM_THRESHOLD", "malloc_trim_threshold")):
            if os.environ.get(var):                # heap-policy A/B (Service.start applies it)
                setattr(cfg, attr, int(os.environ[var]))
        if self.http_probe_bytes >= 0:
            cfg.http_probe_bytes = self.http_probe_bytes
        if self.http_segments > 0:
            cfg.http_segments = self.http_segments
        if self.http_stripe_bytes >= 0:
            cfg.http_stripe_bytes = self.http_stripe_bytes
        if self.s3_part_size > 0:
            cfg.s3_part_size = self.s3_part_size
        if self.s3_multipart_threshold > 0:
            cfg.s3_multipart_threshold = self.s3_multipart_threshold
        if self.sign_threads > 0:
            cfg.s3_sign_threads = self.sign_threads
        for k, v in self.overrides.items():
            setattr(cfg, k, v)
        self.cfg = cfg
        mode = self.payload_mode or ("unsigned" if s3_url.startswith("https://") else "streaming")
        self.payload_mode = mode
        amqp = Client(broker_url, prefetch=self.prefetch, heartbeat=self.heartbeat, retry_delay=0)
        up = Uploader(cfg.bucket, S3Client(s3_url, Static(AK, SK), payload_mode=mode,
                                           sign_threads=cfg.s3_sign_threads, ca_file=cfg.ca_file,
                                           part_size=cfg.s3_part_size, multipart_threshold=cfg.s3_multipart_threshold,
                                           parallel_parts=cfg.s3_parallel_parts, hash_device=self.hash_device))
        self.svc = Service(cfg, amqp=amqp, uploader=up)
        await self.svc.start()
        self.converts: list[Convert] = []
        self._convert_waiter: tuple[int, asyncio.Future] | None = None
        if not producer:
            return
        if not self.inproc:
            # the producing / converting services run in a process of their own, off
            # this worker's event loop (bench_producer.py)
            self.producer_proc = await Backend("producer", [
                "--broker", broker_url, "--origins", ",".join(self.origin_urls), "--size", str(self.file_size),
                "--tag", self.tag, "--broker-pid", str(self.broker_pid),
                "--variants", str(self.resolved_variants())], module="tritondl_testkit.bench_producer").start()
            return
        self.producer = await Connection.open(broker_url, heartbeat=0)
        self.pch = await self.producer.channel()
        await self.pch.confirm_select()
        self.convert_ch = await self.producer.channel()

        def on_convert(m) -> None:
            self.converts.append(Convert.decode(m.body))
            asyncio.ensure_future(m.ack())
            w = self._convert_waiter
            if w is not None and len(self.converts) >= w[0] and not w[1].done():
                w[1].set_result(None)

        # the worker declared v1.convert-{0,1} on its first publish; declare them here too
        for i in range(2):
            await self.convert_ch.queue_declare(f"v1.convert-{i}", durable=True)
        await self.convert_ch.basic_consume("v1.convert-0", on_convert)
        await self.convert_ch.basic_consume("v1.convert-1", on_convert)

    def job_name(self, i: int) -> str:
        r = self.resolved_variants()
        return f"movie-{i}-v{i % r}.mkv" if r else f"movie-{i}.mkv"

    def job_body(self, i: int) -> tuple[str, bytes]:
        mid = f"bench-{self.tag}-{i}"
        origin = self.origin_urls[i % len(self.origin_urls)]
        url = f"{origin}/synthetic/{self.file_size}/{self.job_name(i)}"
        d = Download(created_at="now", media=Media(id=mid, name=f"movie {i}", source=SourceType.HTTP,
                                                      source_uri=url))
        return mid, d.encode()

    async def submit(self, n: int) -> list[str]:
        """Publish n jobs with confirms pipelined (up to 256 outstanding), so
        the producer costs one broker round trip per batch, not per job."""
        ids = []
        pending: list[asyncio.Future] = []
        for _ in range(n):
            i = self._n
            self._n += 1
            mid, body = self.job_body(i)
            fut = await self.pch.basic_publish("v1.download", f"v1.download-{i % 2}", body,
                                               Properties(delivery_mode=2, content_type="application/octet-stream"),
                                               wait_confirm=False)
            if fut is not None:
                pending.append(fut)
            if len(pending) >= 256:
                await asyncio.gather(*pending)
                pending.clear()
            ids.append(mid)
        if pending:
            await asyncio.gather(*pending)
        return ids

    async def wait_done(self, total: int, timeout: float = 600) -> None:
        """Wait (event-driven: no polling on the workers' loop) until the
        worker has finished ``total`` jobs in all."""
        assert self.svc is not None
        await self.svc.wait_finished(total, timeout)

    async def run_jobs(self, n: int) -> float:
        """Submit n jobs and wait for all to finish on THIS worker; returns elapsed seconds."""
        assert self.svc is not None
        base, start = len(self.svc.results), self.svc.jobs_finished
        t0 = time.perf_counter()
        if self.producer_proc is not None:
            self.last_run = await self.producer_proc.request({"cmd": "run", "n": n})
        else:
            await self.submit(n)
        await self.wait_done(start + n)
        dt = time.perf_counter() - t0
        bad = [r for r in self.svc.results[base:] if not r.ok or r.bytes != self.file_size]
        if bad:
            raise RuntimeError(f"{len(bad)} jobs failed: {bad[0]}")
        return dt

    async def run_global(self, n: int, timeout: float = 600) -> float:
        """Producer side of shared mode: submit n jobs for ALL competing workers
        and wait until n new ``v1.convert`` messages arrived (the global ack
        rate's numerator)."""
        if self.producer_proc is not None:
            t0 = time.perf_counter()
            self.last_run = await self.producer_proc.request({"cmd": "run", "n": n, "timeout": timeout})
            return time.perf_counter() - t0
        base = len(self.converts)
        t0 = time.perf_counter()
        fut = asyncio.get_running_loop().create_future()
        self._convert_waiter = (base + n, fut)
        try:
            await self.submit(n)
            if len(self.converts) < base + n:
                await asyncio.wait_for(fut, timeout)
        except asyncio.TimeoutError:
            raise TimeoutError(f"only {len(self.converts) - base}/{n} converts") from None
        finally:
            self._convert_waiter = None
        return time.perf_counter() - t0

    def cpu_seconds(self) -> dict:
        """CPU time (user+sys, s) so far of this worker process (all threads:
        native pumps included; getrusage, microsecond resolution), of its
        event-loop thread (``worker_loop``, when called from it) and pump
        threads, and of this stack's out-of-process fakes (producer included;
        /proc clock ticks, 10 ms resolution)."""
        import resource

        import psutil
        from tritondl.utils import rawhttp
        ru = resource.getrusage(resource.RUSAGE_SELF)
        out = {"worker": ru.ru_utime + ru.ru_stime, "fakes": 0.0, "broker": 0.0, "origin": 0.0, "s3": 0.0,
               "producer": 0.0,
               # the calling thread: the bench runs the worker's event loop on it
               "worker_loop": time.thread_time()}
        # the worker's data-plane pumps, by stage (thread CPU of the executor threads
        # running them; native helper threads they start are in "worker" only)
        for name, key in (("recv_body", "worker_recv"), ("send_body", "worker_send")):
            out[key] = float(rawhttp.PUMP_CPU.get(name, (0.0, 0))[0])
        for b in self.backends + ([self.producer_proc] if self.producer_proc is not None else []):
            p = getattr(b, "proc", None)
            if p is None:
                continue
            try:
                ft = psutil.Process(p.pid).cpu_times()
            except psutil.Error:
                continue
            out["fakes"] += ft.user + ft.system
            kind = "origin" if b.kind == "h2origin" else b.kind
            if kind in out:
                out[kind] += ft.user + ft.system
        return out

    def failures(self) -> list:
        assert self.svc is not None
        return [r for r in self.svc.results if not r.ok or r.bytes != self.file_size]

    async def teardown(self) -> None:
        if self.producer is not None:
            with contextlib.suppress(Exception):
                await self.producer.close()
        if self.producer_proc is not None:
            with contextlib.suppress(Exception):
                await self.producer_proc.stop()
        if self.svc is not None:
            await self.svc.shutdown(grace=10)
        for b in self.backends:
            with contextlib.suppress(Exception):
                await b.stop()
        if self.workdir and os.path.isdir(self.workdir):
            shutil.rmtree(self.workdir, ignore_errors=True)


def run_single_job_smoke(size: int = 1 << 20) -> None:
    """One Download job end-to-end through in-process fakes; asserts the
    Convert message carries the job's Media verbatim and S3 got the bytes."""
    async def main() -> None:
        st = JobStack(file_size=size, inproc=True, tag="smoke")
        await st.setup()
        try:
            await st.run_jobs(1)
            for _ in range(200):
                if st.converts:
                    break
                await asyncio.sleep(0.01)
            assert st.converts, "no v1.convert published"
            c = st.converts[0]
            assert c.media is not None and c.media.id == "bench-smoke-0"
            from .fakes.payload import variant_bytes, variant_of
            s3 = st.backends[-1]
            from tritondl.s3.uploader import object_key
            got = s3.object_bytes("triton-staging", object_key(c.media.id, st.job_name(0)))
            want = variant_bytes(size, variant_of(st.job_name(0)))
            assert hashlib.md5(got).digest() == hashlib.md5(want).digest()
            assert s3.counts["content_ok"] == 1
        finally:
            await st.teardown()
    asyncio.run(asyncio.wait_for(main(), 120))
