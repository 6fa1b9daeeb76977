#!/usr/bin/env python3
"""Flagship benchmark — BASELINE.json config #1:
"Single HTTP download job via local RabbitMQ, 10 MB file".

One *step* = one complete ingest job, exactly as in production: a protobuf
``api.Download`` is published to ``v1.download``; the worker consumes it
(prefetch 1, one job loop — the reference's settings), fetches the 10 MiB
file over HTTP into ``downloading/<id>/``, selects the media file, uploads
it to S3 ``triton-staging/<id>/original/<b64>`` with SigV4 aws-chunked
signing (verified by the fake S3), publishes ``api.Convert`` to
``v1.convert`` (broker-confirmed) and acks.  Broker, origin and S3 are
local fakes, each in its own process; the payload is synthetic.

Multi-GPU (torchrun, one rank per GPU): job-level data parallelism — the
reference's competing consumers (``internal/rabbitmq/client.go:405-422``;
SURVEY.md §2.3).  Rank 0 hosts ONE broker; every rank runs a worker that
competes on the same ``v1.download-{0,1}`` queues, plus its own origin and S3
node (sharded fakes: one single-process fake would cap the node, like one
MinIO disk).  Rank 0 publishes N·K jobs and the timed region ends when N·K
``v1.convert`` messages are back: ``value`` is the global ack rate (N·K /
max-rank elapsed), per-rank work is fixed on average: ``scaling="weak"``.
``--isolated`` restores private per-rank stacks; ``--tls`` runs origin and
S3 over https (OpenSSL in the native data plane).

Every job fetches its own payload variant and the S3 fake refuses a PUT
whose content is not that variant's (64 KiB-leaf SHA-256 list, computed
natively while the chunk signatures are verified): a worker uploading
stale or torn bytes fails the run.  ``config`` states the cleanup mode
(the reference never deletes a job dir, B15) and the spare-file recycling
budget; ``diag`` carries what explains a slow run (per-job latency spread,
CCD load at launch, CPU clocks, faults and context switches per job,
whether this was the lease's first run).

The reference publishes no numbers → ``vs_baseline: null``.
A secondary, untimed-for-headline figure reports the HIP batched piece-hash
kernel (torrent resume verification) on this GPU.
"""

from __future__ import annotations

import argparse
import asyncio
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIG_NAME = "Single HTTP download job via local RabbitMQ, 10 MB file"


def _gpu_hash_probe(total_mb: int = 4096) -> dict:
    """Secondary metric: HIP SHA-1 piece kernel on device-resident data.  One
    lane hashes one piece, so the buffer is sized for the 256 KiB figure to
    fill the device: 4 GiB = 16,384 pieces (262,144 at 16 KiB); the lane
    count is reported with each rate."""
    try:
        import torch

        from tritondl.ops import hashing
        if not (torch.cuda.is_available() and hashing.gpu_available()):
            return {}
        mod = hashing.gpu_module()
        total = total_mb << 20
        dev = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
        out = {}
        for pk in (16, 256):
            pl = pk << 10
            n = total // pl
            o = torch.empty(n * 20, dtype=torch.uint8, device="cuda")
            s = torch.cuda.current_stream().cuda_stream
            mod.hash_device("sha1", dev.data_ptr(), total, pl, o.data_ptr(), s)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps = 5
            for _ in range(reps):
                mod.hash_device("sha1", dev.data_ptr(), total, pl, o.data_ptr(), s)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            out[f"gpu_sha1_piece{pk}k_GBps"] = round(total / dt / 1e9, 1)
            out[f"gpu_sha1_piece{pk}k_lanes"] = n
        del dev
        torch.cuda.empty_cache()
        return out
    except Exception as e:  # secondary figure only
        return {"gpu_probe_error": str(e)[:200]}


_PLACEMENT: dict = {}


def _memcpy_gbps(mb: int = 64, reps: int = 4) -> float | None:
    """Single-thread copy bandwidth on this rank's CPUs (best of ``reps``
    copies of ``mb`` MiB, GB/s of bytes copied): a co-tenant saturating the
    socket's memory shows up here, where CCD busy shares do not."""
    try:
        import numpy as np
        a = np.ones(mb << 20, dtype=np.uint8)
        b = np.empty_like(a)
        best = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            np.copyto(b, a)
            best = min(best, time.perf_counter() - t0)
        return round(a.nbytes / best / 1e9, 1)
    except Exception:  # noqa: BLE001 - diagnostics only
        return None


_VMSTAT = ("nr_dirtied", "nr_written", "allocstall_normal", "allocstall_movable", "pgscan_direct",
           "compact_stall", "workingset_refault_file", "pgfault")


def _vm_snapshot() -> dict:
    """Host page-cache state: selected ``/proc/vmstat`` counters and the
    Dirty / Writeback totals of ``/proc/meminfo`` (kB).  Writeback by other
    tenants and direct reclaim both stall a download's page-cache writes."""
    out: dict = {}
    try:
        with open("/proc/vmstat") as f:
            for line in f:
                k, _, v = line.partition(" ")
                if k in _VMSTAT:
                    out[k] = int(v)
        with open("/proc/meminfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                if k in ("Dirty", "Writeback"):
                    out[k + "_kB"] = int(v.split()[0])
    except (OSError, ValueError):
        pass
    return out


def _vm_delta(v0: dict, v1: dict, n: int) -> dict:
    """Per-job vmstat deltas plus the start/end Dirty and Writeback totals.
    These are HOST-wide counters (every process on the machine, the fakes and
    other tenants included); the worker's own faults are ``minflt_per_job``."""
    out: dict = {k + "_per_job": round((v1[k] - v0[k]) / max(1, n), 1) for k in _VMSTAT if k in v0 and k in v1}
    out["scope"] = "host"
    for k in ("Dirty_kB", "Writeback_kB"):
        if k in v0 and k in v1:
            out[k] = [v0[k], v1[k]]
    return out


def _work_fs(stack) -> dict | None:
    """Filesystem of the worker's download dir, and its spare-file pool's use."""
    try:
        from tritondl.check import mount_of
        from tritondl.utils import spares
        d = stack.cfg.download_dir
        out = mount_of(d)
        pool = spares.pool_for(os.path.join(d, "x"))
        if pool is not None:
            out["spares_taken"], out["spares_offered"] = pool.taken, pool.offered
        return out
    except Exception:  # noqa: BLE001 - diagnostics only
        return None


def _cpu_mhz(cpus: list[int]) -> dict | None:
    """Current clock of the given CPUs (cpufreq, else /proc/cpuinfo): min/mean/max MHz."""
    vals: list[float] = []
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cpufreq/scaling_cur_freq") as f:
                vals.append(int(f.read()) / 1000.0)
        except (OSError, ValueError):
            vals = []
            break
    if not vals:
        try:
            mhz: dict[int, float] = {}
            cur = -1
            with open("/proc/cpuinfo") as f:
                for line in f:
                    if line.startswith("processor"):
                        cur = int(line.split(":")[1])
                    elif line.startswith("cpu MHz") and cur >= 0:
                        mhz[cur] = float(line.split(":")[1])
            vals = [mhz[c] for c in cpus if c in mhz]
        except (OSError, ValueError):
            return None
    if not vals:
        return None
    return {"min": round(min(vals)), "mean": round(sum(vals) / len(vals)), "max": round(max(vals)), "n": len(vals)}


def _lease_state() -> dict:
    """Was this the first bench on this host since it booted / was leased?  A
    marker in /tmp (fresh on every gpurun box) says; uptime and load help."""
    import tempfile
    marker = os.path.join(tempfile.gettempdir(), "tritondl-bench-ran")
    fresh = not os.path.exists(marker)
    try:
        with open(marker, "a") as f:
            f.write(f"{time.time()}\n")
    except OSError:
        pass
    out: dict = {"lease_fresh": fresh}
    try:
        with open("/proc/uptime") as f:
            out["host_uptime_s"] = round(float(f.read().split()[0]))
        out["loadavg"] = [round(x, 2) for x in os.getloadavg()]
    except (OSError, ValueError):
        pass
    return out


def _trace_p50(events: list) -> dict:
    """p50 offset (ms) of each data-plane event from its job's ``job_start``
    (``TRITONDL_TRACE=1``; meaningful at concurrency 1, where a job's events
    follow its start)."""
    per: dict[str, list[float]] = {}
    start = None
    for name, t in events:
        if name == "job_start":
            start = t
            continue
        if start is not None:
            per.setdefault(name, []).append((t - start) * 1000)
    return {k: round(sorted(v)[len(v) // 2], 3) for k, v in sorted(per.items(), key=lambda kv: sorted(kv[1])[0])}


_CPU_KEYS = ("worker", "worker_loop", "worker_recv", "worker_send", "fakes", "origin", "s3", "broker", "producer")


def _cpu_per_job(cpu_all: list, jobs: int) -> dict:
    return {k: round(sum(c.get(k, 0.0) for c in cpu_all) / max(1, jobs) * 1000, 3) for k in _CPU_KEYS}


# Run-to-run spread of this bench in the driver's form (--steps 20 --warmup 5), measured by
# the builder on MI355X boxes (profiles/r06_noise/SUMMARY.md).  One run's number moves this much
# between back-to-back runs on one box: a change smaller than it is not resolved by one record.
BUILDER_SPREAD = {"form": "--steps 20 --warmup 5", "runs": 6, "concurrency": 1,
                  "jobs_per_sec": [385.6, 411.5, 408.1, 419.9, 402.9, 393.5], "mean": 403.6, "stdev": 11.4,
                  "range_pct_of_mean": 8.5,
                  # 26 driver-form runs of the late round-6 trees on several boxes, co-tenant load
                  # included (profiles/r06_final4/, r06_final5/): the tail is the host, not the tree
                  "late_trees": {"runs": 26, "median": 380.2, "mean": 363.6, "stdev": 46.2, "min": 238.1,
                                 "max": 411.3, "runs_below_310": 5}}


def _noise(done: list, lat: list) -> dict:
    """How much to trust one run's number: the per-job latency IQR, the job
    rate of each quarter of the timed jobs (by completion time), and the
    run-to-run spread of this bench measured by the builder on the MI355X
    boxes (:data:`BUILDER_SPREAD`)."""
    out: dict = {}
    if lat:
        q = lambda f: round(lat[min(len(lat) - 1, int(len(lat) * f))] * 1000, 3)  # noqa: E731
        out["latency_ms_p25_p75"] = [q(0.25), q(0.75)]
        out["latency_ms_iqr"] = round(q(0.75) - q(0.25), 3)
    ts = [r.finished_at for r in done if getattr(r, "finished_at", 0.0)]
    if len(ts) >= 8:
        k = len(ts) // 4
        rates = []
        for i in range(4):
            seg = ts[i * k:(i + 1) * k + 1] if i < 3 else ts[3 * k:]
            if len(seg) >= 2 and seg[-1] > seg[0]:
                rates.append(round((len(seg) - 1) / (seg[-1] - seg[0]), 1))
        if len(rates) == 4:
            out["quarter_jobs_per_sec"] = rates
            out["quarter_spread_pct"] = round((max(rates) - min(rates)) / (sum(rates) / 4) * 100, 1)
    out["builder_run_to_run"] = BUILDER_SPREAD
    return out


def _place(cpus: str, fake_cpus: str, local_rank: int, local_world: int, file_size: int) -> list[int]:
    """Pin this rank's process (inherited by every native thread and by the
    fakes it spawns) before anything starts, and choose the fakes' set.

    ``auto``: each rank gets whole L3 domains, one for small jobs and two for
    jobs of 256 MiB and up (a 1 GiB job's ~9 CPUs of pump and hashing work
    does not fit one CCD: 7.7-8.4 jobs/s on one, 9.8-12.3 on two,
    ``profiles/r03_place_ab2/``); the fakes, which stand in for remote
    endpoints, get one more domain on the rank's NUMA node (``--fake-cpus
    auto``, ``topology.pair_domains``), so on a 16-CCD node 8 ranks and their
    fakes pair up within the sockets.  Domains are taken idle-first (sampled
    once per launch by local rank 0): a shared host's busy CCDs go last."""
    from tritondl.parallel import topology
    fc: list[int] = []
    pinned: list[int] = []
    # before pinning (afterwards only our own CPUs show), and idle-first: on a host
    # shared with other tenants a fixed CCD 0..n can be one they keep busy
    # (profiles/r03_final4/: ranks on CCDs 2-5 did 125-168 jobs against 208-256)
    tag = f"{os.getppid()}-{os.environ.get('MASTER_PORT', '0')}"
    doms, busy = (topology.shared_idle_order(local_rank, local_world, tag) if cpus == "auto"
                  else (topology.l3_domains(), []))
    k = 2 if file_size >= 256 << 20 else 1
    # with room for it, every rank gets k domains and its fakes one more, all on one
    # NUMA node (the idle ranking alone can put the fakes across the socket:
    # topology.pair_domains); otherwise the ranks come first and the fakes after them all
    pairs = topology.pair_domains(doms, k, local_world) if cpus == "auto" else None
    packed = len(doms) >= (k + 1) * local_world
    first = local_rank * (k + 1) if packed else local_rank * k
    if fake_cpus not in ("", "same") and cpus not in ("", "none"):
        if fake_cpus != "auto":
            fc = topology.parse_cpulist(fake_cpus)
        elif pairs is not None:
            fc = pairs[local_rank][1]
        else:
            fc = doms[(first + k if packed else local_world * k + local_rank) % len(doms)]
    if cpus == "auto":
        mine = pairs[local_rank][0] if pairs is not None else [doms[(first + j) % len(doms)] for j in range(k)]
        pinned = sorted({c for d in mine for c in d})
        os.sched_setaffinity(0, pinned)
        if busy:
            share = dict(zip((d[0] for d in doms), busy))
            os.environ["TRITONDL_BENCH_DOMAIN_BUSY"] = f"{share[mine[0][0]]:.2f}"
            # every L3 domain's busy share at launch, in topology order (first CPU: share)
            _PLACEMENT["ccd_busy_at_launch"] = {str(c): round(b, 3) for c, b in sorted(share.items())}
            _PLACEMENT["chosen_ccds"] = sorted(d[0] for d in mine)
        if fc:
            _PLACEMENT["fake_ccd"] = fc[0]
            _PLACEMENT["fakes_same_numa_node"] = topology.numa_node_of(fc[0]) == topology.numa_node_of(pinned[0])
    elif cpus not in ("", "none"):
        pinned = topology.pin(cpus, local_rank)
    if fc:
        os.environ["TRITONDL_BENCH_FAKE_CPUS"] = ",".join(map(str, fc))
    return pinned


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--file-mb", type=float, default=10.0)
    ap.add_argument("--concurrency", type=int, default=0,
                    help="jobs in flight per worker: 0 = the worker default (adaptive, 1..4), N = fixed "
                         "(reference: 1)")
    ap.add_argument("--prefetch", type=int, default=0, help="AMQP prefetch per shard consumer (0: = concurrency)")
    ap.add_argument("--no-gpu-probe", action="store_true")
    ap.add_argument("--probe-kb", type=int, default=-1,
                    help="HTTP GET probe size in KiB, the rest as parallel Range streams "
                         "(-1: worker default, 0: open-ended probe)")
    ap.add_argument("--http-segments", type=int, default=0, help="max parallel Range streams (0: worker default)")
    ap.add_argument("--segment-threshold-mb", type=float, default=0,
                    help="files at least this big are fetched as parallel Range streams (0: worker default)")
    ap.add_argument("--s3-part-mb", type=int, default=0, help="S3 multipart part size (0: worker default)")
    ap.add_argument("--s3-parallel-parts", type=int, default=0, help="S3 parts in flight per file (0: worker default)")
    ap.add_argument("--s3-multipart-mb", type=int, default=0,
                    help="objects at least this big go multipart (0: worker default, 64 MiB like minio-go)")
    ap.add_argument("--stripe-kb", type=int, default=-1,
                    help="parallel streams pull in-order stripes of this size (-1: worker default, 0: off)")
    ap.add_argument("--sign-threads", type=int, default=0, help="S3 chunk hashers per PUT (0: worker default)")
    ap.add_argument("--tls", action="store_true", help="origin and S3 over https (self-signed CA)")
    ap.add_argument("--payload", default="", choices=["", "streaming", "unsigned"],
                    help="S3 payload mode ('' = aws-chunked over http, unsigned over https, like minio-go)")
    ap.add_argument("--isolated", action="store_true",
                    help="multi-rank: every rank gets a private broker (default: one shared broker, "
                         "competing consumers)")
    ap.add_argument("--dist-backend", default="", help="torch.distributed backend (default nccl with a GPU)")
    ap.add_argument("--dist-always", action="store_true",
                    help="set up torch.distributed (RCCL with a GPU) and do the closing max-reduce over it even "
                         "for one rank: exercises the multi-GPU path's collectives on a one-GPU box")
    ap.add_argument("--log-level", default="warning")
    ap.add_argument("--s3-hash-device", default="cpu", choices=["cpu", "gpu"],
                    help="aws-chunked chunk SHA-256s on SHA-NI (default) or the HIP kernel")
    ap.add_argument("--cpuprofile", default="",
                    help="sampled whole-process CPU profile of the timed region (pprof + .txt summary; "
                         "rank r writes PATH.r<r> when N > 1)")
    ap.add_argument("--cpus", default="auto",
                    help="pin this rank (worker, fakes, pump threads) to a CPU set: a cpulist like 0-15, "
                         "auto = whole L3 domains (CCD + SMT siblings) per rank: one, or two for files "
                         "of 256 MiB and up; auto:N = N CPUs "
                         "packed into the fewest L3 domains; 'none' = no pinning.  Default auto: on the "
                         "16-CPU box share one CCD measured 323-336 vs 222-279 jobs/s unpinned, "
                         "profiles/r03_pin_ab/)")
    ap.add_argument("--cleanup", default="on", choices=["on", "off"],
                    help="on (the worker default): each settled job's dir is deleted (its file kept as a spare "
                         "the next download is renamed into, up to --recycle-mb); off: the reference, which never "
                         "deletes (B15)")
    ap.add_argument("--recycle-mb", type=int, default=-1, help="spare-file budget with cleanup on (-1: worker "
                                                               "default, 0: delete every file)")
    ap.add_argument("--variants", type=int, default=-1,
                    help="distinct payloads jobs rotate through (-1: more than the spare pool holds)")
    ap.add_argument("--pipeline-min-ms", type=float, default=-1.0,
                    help="pipeline commits only while the confirm round trip is at least this (ms; -1: worker default)")
    ap.add_argument("--pipeline-commit", default="on", choices=["on", "off"],
                    help="on (the worker default): a job's publish confirm and ack overlap the next job")
    ap.add_argument("--lease-after", type=float, default=-1.0,
                    help="lease a job's delivery once it has run this long (s; -1: worker default 30 s, which a "
                         "10 MiB job never reaches; a tiny value leases every job, to price the lease)")
    ap.add_argument("--h2-origin", action="store_true",
                    help="with --tls: the fake origin serves HTTP/2 (ALPN h2; Python frames) instead of HTTP/1.1")
    ap.add_argument("--http2", default="default", choices=["default", "on", "off"],
                    help="offer HTTP/2 to https origins (default: the worker's, on); matters with --tls only")
    ap.add_argument("--no-reference-mode", action="store_true",
                    help="skip the secondary run in the reference's cleanup-off mode after the timed region")
    ap.add_argument("--no-content-check", action="store_true",
                    help="S3 does not compare PUT content with the origin's payload")
    ap.add_argument("--rtt-ms", type=float, default=0.0,
                    help="emulated network round trip of the fake broker / origin / S3 (ms): every new "
                         "connection, TLS handshake, request/response and broker frame waits one RTT "
                         "(a latency model; loopback bandwidth).  0 = loopback, the headline")
    ap.add_argument("--stream-mbps", type=float, default=0.0,
                    help="cap each origin response / S3 PUT stream of the fakes at this many Mbit/s (one TCP "
                         "stream's window / RTT on a real path); 0 = uncapped, the headline")
    ap.add_argument("--fake-cpus", default="auto",
                    help="pin the fake broker/origin/S3/producer processes (remote endpoints in "
                         "production) elsewhere: a cpulist, auto = the L3 domain after the last rank's, "
                         "'same' = the rank's own set")
    a = ap.parse_args()
    lease = _lease_state()
    if a.rtt_ms > 0:
        os.environ["TRITONDL_FAKE_RTT_MS"] = str(a.rtt_ms)   # the fake processes inherit it
    if a.stream_mbps > 0:
        os.environ["TRITONDL_FAKE_STREAM_MBPS"] = str(a.stream_mbps)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    try:
        pinned = _place(a.cpus, a.fake_cpus, local_rank, int(os.environ.get("LOCAL_WORLD_SIZE", world)),
                        int(a.file_mb * 1024 * 1024))
    except (OSError, ValueError, IndexError) as e:     # placement is an optimisation: run unpinned
        print(f"bench: CPU placement skipped ({e})", file=sys.stderr, flush=True)
        os.environ.pop("TRITONDL_BENCH_FAKE_CPUS", None)
        pinned = []

    import torch
    import torch.distributed as dist

    backend = a.dist_backend or ("nccl" if torch.cuda.is_available() else "gloo")
    cuda = torch.cuda.is_available() and backend == "nccl"
    if cuda:
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    ctl = None
    use_dist = world > 1 or a.dist_always
    if use_dist:
        import datetime
        # a collective that cannot complete aborts the run in minutes, not at the driver's limit
        dist.init_process_group(backend, timeout=datetime.timedelta(minutes=5))
        # control plane (endpoint exchange, phase barriers from a helper thread): gloo
        ctl = dist.new_group(backend="gloo") if backend != "gloo" else dist.group.WORLD
    shared = world > 1 and not a.isolated

    def barrier() -> None:
        if use_dist:
            dist.barrier(group=ctl)
        if cuda:
            torch.cuda.synchronize()

    from tritondl_testkit.bench_job import JobStack
    from tritondl.utils.log import log
    log.configure(a.log_level, "")

    file_size = int(a.file_mb * 1024 * 1024)
    prefetch = a.prefetch if a.prefetch > 0 else max(1, a.concurrency)
    stack = JobStack(file_size=file_size, concurrency=a.concurrency, prefetch=prefetch,
                     tag=f"r{rank}", http_probe_bytes=(a.probe_kb << 10) if a.probe_kb >= 0 else -1,
                     http_segments=a.http_segments, sign_threads=a.sign_threads, tls=a.tls,
                     h2_origin=a.h2_origin,
                     http_stripe_bytes=(a.stripe_kb << 10) if a.stripe_kb >= 0 else -1,
                     s3_part_size=a.s3_part_mb << 20, s3_multipart_threshold=a.s3_multipart_mb << 20,
                     payload_mode=a.payload, hash_device=a.s3_hash_device, cleanup=a.cleanup == "on",
                     recycle_bytes=(a.recycle_mb << 20) if a.recycle_mb >= 0 else -1, variants=a.variants,
                     content_check=not a.no_content_check,
                     overrides={"pipeline_commit": a.pipeline_commit == "on",
                                **({"lease_after_s": a.lease_after} if a.lease_after >= 0 else {}),
                                **({"http2": a.http2 == "on"} if a.http2 != "default" else {}),
                                **({"pipeline_commit_min_ms": a.pipeline_min_ms} if a.pipeline_min_ms >= 0 else {}),
                                **({"http_segment_threshold": int(a.segment_threshold_mb * (1 << 20))}
                                   if a.segment_threshold_mb > 0 else {}),
                                **({"s3_parallel_parts": a.s3_parallel_parts} if a.s3_parallel_parts > 0 else {})})
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)

    async def phase(n_per_rank: int) -> None:
        """Shared mode: rank 0 publishes world*n jobs and waits for as many
        v1.convert messages; every rank's worker competes for them until the
        closing barrier (run off-loop so the workers keep working)."""
        if rank == 0:
            await stack.run_global(world * n_per_rank)
        await loop.run_in_executor(None, lambda: dist.barrier(group=ctl))

    try:
        if shared:
            mine = loop.run_until_complete(stack.start_backends(broker=rank == 0))
            ca_pem = ""
            if a.tls:
                with open(mine["ca_file"]) as f:
                    ca_pem = f.read()
            gathered: list = [None] * world
            dist.all_gather_object(gathered, {**mine, "ca_pem": ca_pem}, group=ctl)
            endpoints = {"broker": gathered[0]["broker"], "origin": mine["origin"], "s3": mine["s3"]}
            if a.tls:   # every rank trusts every rank's throwaway CA (origins are shared)
                both = os.path.join(stack.workdir, "all-ca.pem")
                with open(both, "w") as f:
                    f.write("".join(g["ca_pem"] for g in gathered))
                endpoints["ca_file"] = both
            loop.run_until_complete(stack.setup(endpoints, origins=[g["origin"] for g in gathered],
                                                producer=rank == 0))
        else:
            loop.run_until_complete(stack.setup())
        c = stack.cfg
        knobs = ({"http_probe_bytes": c.http_probe_bytes, "http_segments": c.http_segments,
                  "http_stripe_bytes": c.http_stripe_bytes, "s3_sign_threads": c.s3_sign_threads,
                  "s3_part_size": c.s3_part_size, "s3_multipart_threshold": c.s3_multipart_threshold,
                  "s3_parallel_parts": c.s3_parallel_parts}
                 if c is not None else {})
        # probes that touch a lot of memory or import modules run BEFORE the
        # warm-up: between warm-up and the timed region they evicted the
        # caches the first timed job runs from (first job 4.4 vs 2.5 ms p50)
        stack.cpu_seconds()              # first call imports psutil: keep it out of the timed window
        mem0 = _memcpy_gbps()
        cpu_w0 = stack.cpu_seconds()     # warm-up + timed window (fakes' /proc ticks are 10 ms)
        if a.warmup:
            if shared:
                loop.run_until_complete(phase(a.warmup))
            else:
                loop.run_until_complete(stack.run_jobs(a.warmup))
        start = stack.svc.jobs_finished  # type: ignore[union-attr]
        prof = None
        if a.cpuprofile:
            from tritondl.utils.profiler import CPUProfiler
            prof = CPUProfiler(a.cpuprofile if world == 1 else f"{a.cpuprofile}.r{rank}")
        import resource
        mhz0 = _cpu_mhz(pinned) if pinned else None
        vm0 = _vm_snapshot()
        barrier()
        if prof is not None:
            prof.start()
        # diagnostic: deterministic profile of the event-loop thread's own CPU
        # (thread_time clock) over the timed jobs only
        loop_prof = None
        if os.environ.get("TRITONDL_BENCH_LOOP_PROFILE"):
            import cProfile
            loop_prof = cProfile.Profile(time.thread_time)
            loop_prof.enable()
        cpu0 = stack.cpu_seconds()
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        gc0 = [g["collections"] for g in gc.get_stats()]
        from tritondl.utils import rawhttp as _rh
        if _rh.TRACE is not None:
            _rh.TRACE.clear()               # TRITONDL_TRACE=1: data-plane events of the timed jobs only
        t0 = time.perf_counter()
        if shared:
            loop.run_until_complete(phase(a.steps))
        else:
            loop.run_until_complete(stack.run_jobs(a.steps))
        if cuda:
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        svc = stack.svc
        conc = {"limit": svc._limit, "changes": int(svc.metrics.get("concurrency_changes")),
                "last_decision": svc._adapt.last if svc._adapt is not None else None}
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        gc1 = [g["collections"] for g in gc.get_stats()]
        vm1 = _vm_snapshot()
        cpu1 = stack.cpu_seconds()
        mhz1 = _cpu_mhz(pinned) if pinned else None
        mem1 = _memcpy_gbps()
        if loop_prof is not None:
            loop_prof.disable()
            loop_prof.dump_stats(os.environ["TRITONDL_BENCH_LOOP_PROFILE"])
        if prof is not None:
            prof.stop()
        barrier()
        n_done = stack.svc.jobs_finished - start  # type: ignore[union-attr]
        # latency/span stats over the recent-results window (trimmed past 10,000)
        done = stack.svc.results[-n_done:] if n_done else []  # type: ignore[union-attr]
        failed = len(stack.failures())
        lat = sorted(r.seconds for r in done)
        n_div = max(1, n_done)
        diag = {**lease, **_PLACEMENT,
                "job_latency_ms": ({"min": round(lat[0] * 1000, 2), "max": round(lat[-1] * 1000, 2),
                                    "first": round(done[0].seconds * 1000, 2),
                                    "first_marks": {k: round(v * 1000, 2) for k, v in done[0].marks.items()},
                                    "last": round(done[-1].seconds * 1000, 2)} if done else None),
                "cpu_mhz_pinned": {"start": mhz0, "end": mhz1},
                "memcpy_GBps": {"start": mem0, "end": mem1},
                # jobs slower than 3x the median (and 10 ms): index in the timed run, ms, stage marks
                "slow_jobs": ([{"i": i, "ms": round(r.seconds * 1000, 1),
                                "marks": {k: round(v * 1000, 1) for k, v in r.marks.items()}}
                               for i, r in enumerate(done)
                               if r.seconds > max(0.010, 3 * lat[len(lat) // 2])][:8] if done else []),
                "slow_jobs_total_ms": round(sum(r.seconds for r in done
                                                if r.seconds > max(0.010, 3 * lat[len(lat) // 2])) * 1000, 1)
                if done else 0.0,
                # worker process (this rank), per timed job
                "minflt_per_job": round((ru1.ru_minflt - ru0.ru_minflt) / n_div, 1),
                "majflt_per_job": round((ru1.ru_majflt - ru0.ru_majflt) / n_div, 2),
                "nvcsw_per_job": round((ru1.ru_nvcsw - ru0.ru_nvcsw) / n_div, 1),
                "nivcsw_per_job": round((ru1.ru_nivcsw - ru0.ru_nivcsw) / n_div, 1),
                "s3_content_checked": bool(stack.content_check and stack.resolved_variants()),
                "h2_streams": sum(getattr(i, "h2_streams", 0) for i in getattr(stack.svc.dispatcher, "impls", [])
                                  or []) if stack.svc is not None else None,
                "vm": _vm_delta(vm0, vm1, n_div),
                # CPython collections per generation inside the timed region (the worker
                # froze its start-up heap: Service.start -> freeze_startup_heap)
                "gc_collections": {f"gen{i}": b - a for i, (a, b) in enumerate(zip(gc0, gc1))},
                **({"trace_p50_ms": _trace_p50(_rh.TRACE)} if _rh.TRACE else {}),
                "gc_frozen": gc.get_freeze_count(),
                "concurrency": conc,
                "work_fs": _work_fs(stack)}
        noise = _noise(done, lat)
        spans: dict[str, list[float]] = {}
        for r in done:
            for k, v in r.marks.items():
                spans.setdefault(k, []).append(v)
        # secondary, after the headline's timed region: the same jobs in the
        # reference's mode (cleanup off: every job dir kept, fresh files, B15)
        reference_mode = None
        if world == 1 and stack.cleanup and not a.no_reference_mode and stack.svc is not None:
            stack.svc.cfg.cleanup = False
            loop.run_until_complete(stack.run_jobs(max(a.warmup, 5)))   # drains the spare pool (4 files)
            s0 = stack.svc.jobs_finished
            vr0 = _vm_snapshot()
            t0r = time.perf_counter()
            loop.run_until_complete(stack.run_jobs(a.steps))
            dtr = time.perf_counter() - t0r
            vr1 = _vm_snapshot()
            done_r = stack.svc.results[-(stack.svc.jobs_finished - s0):]
            lat_r = sorted(r.seconds for r in done_r)
            fet_r = sorted(r.marks["fetched"] for r in done_r if "fetched" in r.marks)
            reference_mode = {"cleanup": False, "jobs_per_sec": round(a.steps / dtr, 3),
                              "ms_per_step": round(dtr / a.steps * 1000, 3),
                              "job_latency_ms_p50": round(lat_r[len(lat_r) // 2] * 1000, 2) if lat_r else None,
                              "fetched_ms_p50": round(fet_r[len(fet_r) // 2] * 1000, 2) if fet_r else None,
                              "vm": _vm_delta(vr0, vr1, len(done_r)),
                              "steps": a.steps, "warmup": max(a.warmup, 5)}
    finally:
        loop.run_until_complete(stack.teardown())
        loop.close()

    t = torch.tensor([elapsed, float(failed)], dtype=torch.float64, device="cuda" if cuda and use_dist else "cpu")
    if use_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)        # RCCL on the GPU node
    max_elapsed = float(t[0].item())
    if int(t[1].item()):
        raise SystemExit(f"{int(t[1].item())} jobs failed on some rank")
    per_rank = [n_done]
    cpu = {k: cpu1[k] - cpu0[k] for k in cpu0}
    cpu_w = {k: cpu1[k] - cpu_w0[k] for k in cpu_w0}
    cpu_all = [cpu]
    cpu_w_all = [cpu_w]
    if world > 1:
        per_rank = [None] * world  # type: ignore[list-item]
        dist.all_gather_object(per_rank, n_done, group=ctl)
        cpu_all = [None] * world  # type: ignore[list-item]
        dist.all_gather_object(cpu_all, cpu, group=ctl)
        cpu_w_all = [None] * world  # type: ignore[list-item]
        dist.all_gather_object(cpu_w_all, cpu_w, group=ctl)
        # where every rank ran: its CCD(s), its fakes' CCD, one NUMA node or not, memory bandwidth
        mine = {"ccds": _PLACEMENT.get("chosen_ccds"), "fake_ccd": _PLACEMENT.get("fake_ccd"),
                "same_numa_node": _PLACEMENT.get("fakes_same_numa_node"),
                "memcpy_GBps_start": diag["memcpy_GBps"]["start"]}
        placement_all = [None] * world  # type: ignore[list-item]
        dist.all_gather_object(placement_all, mine, group=ctl)
        diag["placement_per_rank"] = placement_all
    extra = {} if (a.no_gpu_probe or rank != 0) else _gpu_hash_probe()
    if rank == 0:
        jobs_per_sec = world * a.steps / max_elapsed
        name = CONFIG_NAME if file_size == 10 << 20 else \
            f"Single HTTP download job via local RabbitMQ, {file_size / 2**20:g} MiB file"
        res = {
            "metric": "jobs_per_sec",
            "value": round(jobs_per_sec, 3),
            "unit": "jobs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(max_elapsed / a.steps * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8",
            "data": f"synthetic ({stack.resolved_variants() or 1} distinct deterministic pseudo-random "
                    f"{file_size / 2**20:g} MiB payloads, one per job in rotation, S3 content-checked; "
                    f"local fake broker/origin/S3{' over https' if a.tls else ''})",
            "config": {"model": name, "global_batch": world * (a.concurrency or 1), "seq_len": None,
                       "file_bytes": file_size, "parallelism": f"dp{world}",
                       "topology": ("one shared broker, competing consumers; per-rank origin+S3 nodes"
                                    if shared else "private broker/origin/S3 per rank"),
                       "transport": ("https, HTTP/2 origin (TLS 1.3, native session pump)" if a.tls and a.h2_origin
                                     else "https (TLS 1.3, native OpenSSL data plane)" if a.tls else "http"),
                       "s3_payload": stack.payload_mode, "s3_hash_device": a.s3_hash_device,
                       "cpus": (f"{len(pinned)} pinned ({pinned[0]}..{pinned[-1]})" if pinned else "unpinned"),
                       "fake_cpus": os.environ.get("TRITONDL_BENCH_FAKE_CPUS", "") or "same as the rank",
                       "cpus_busy_before": os.environ.get("TRITONDL_BENCH_DOMAIN_BUSY", ""),
                       "concurrency_per_worker": a.concurrency or "adaptive",
                       "concurrency_limit_end": conc["limit"],
                       "prefetch": prefetch,
                       "cleanup": stack.cleanup, "pipeline_commit": a.pipeline_commit == "on",
                       "rtt_ms": a.rtt_ms, "stream_mbps": a.stream_mbps or None,
                       "lease_after_s": stack.cfg.lease_after_s if stack.cfg is not None else None,
                       "http2": stack.cfg.http2 if stack.cfg is not None else None,
                       "log_level": a.log_level,
                       "recycle_bytes": stack.resolved_recycle_bytes() if stack.cleanup else 0,
                       "payload_variants": stack.resolved_variants(),
                       "malloc_policy": stack.svc.malloc_policy if stack.svc is not None else {},
                       # the closing max-reduce (RCCL on GPU nodes) and the gloo control group
                       "collectives": (f"{backend} max-reduce + gloo control" if use_dist else "none (one rank)"),
                       **knobs},
            "jobs_per_rank": per_rank,
            "ingest_MB_per_sec": round(jobs_per_sec * file_size / 1e6, 1),
            "job_latency_ms_p50": round(lat[len(lat) // 2] * 1000, 2) if lat else None,
            "job_latency_ms_p90": round(lat[int(len(lat) * 0.9)] * 1000, 2) if lat else None,
            # median ms from taking the job to the end of each stage (rank 0)
            "job_spans_ms_p50": {k: round(sorted(v)[len(v) // 2] * 1000, 2) for k, v in spans.items()},
            # CPU cost per job over the timed region, all ranks (worker processes incl. their
            # native pump threads, from getrusage, microsecond resolution; the out-of-process
            # fakes, producer included, from /proc at 10 ms ticks: read those over a short run
            # as +-10 ms / steps).  The node's CPU count divided by "worker" bounds how far
            # job-level data parallelism can scale.  worker_loop / worker_recv / worker_send:
            # the event-loop thread and the download / upload pump threads (parts of
            # "worker"); origin / s3 / broker / producer: each fake process (parts of "fakes")
            "cpu_ms_per_job": _cpu_per_job(cpu_all, world * a.steps),
            # the same over warm-up + timed jobs (a window long enough for the fakes' ticks)
            "cpu_ms_per_job_with_warmup": _cpu_per_job(cpu_w_all, world * (a.steps + a.warmup)),
            "cpu_window_s": {"timed": round(max_elapsed, 4), "fakes_tick_ms": 10},
            # share of one core each fake process used over the timed region (rank 0's): a
            # fake near 1.0 on a one-job-at-a-time run is what bounds it, not the worker
            "fake_core_share": {k: round(cpu_all[0].get(k, 0.0) / max_elapsed, 3)
                                for k in ("origin", "s3", "broker", "producer")},
            # the one fake broker serves every rank: the share of a core it used.  Above
            # 0.5 the harness, not the workers, may be what limits the run
            "broker_core_share": round(cpu_all[0]["broker"] / max_elapsed, 3),
            "noise": noise,
            "diag": diag,
        }
        if reference_mode is not None:
            # not the number of record: timed after it, with the reference's cleanup-off mode
            res["reference_mode"] = reference_mode
        if res["broker_core_share"] is not None and res["broker_core_share"] > 0.5:
            res["harness_bound"] = True
        res.update(extra)
        print(json.dumps(res), flush=True)
    if use_dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
