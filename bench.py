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

Multi-GPU (torchrun, one rank per GPU): each rank is an independent worker
with its own local backends — job-level data parallelism (competing-consumer
workers) — so per-rank work is fixed: ``scaling="weak"``.
``value`` = total jobs/s over all ranks (N·K / max-rank elapsed).

The reference publishes no numbers → ``vs_baseline: null``.
A secondary, untimed-for-headline figure reports the HIP batched piece-hash
kernel (torrent resume verification) on this GPU.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIG_NAME = "Single HTTP download job via local RabbitMQ, 10 MB file"


def _gpu_hash_probe(total_mb: int = 256) -> dict:
    """Secondary metric: HIP SHA-1 piece kernel on device-resident data."""
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
        return out
    except Exception as e:  # secondary figure only
        return {"gpu_probe_error": str(e)[:200]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--file-mb", type=float, default=10.0)
    ap.add_argument("--concurrency", type=int, default=1, help="jobs in flight per worker (reference: 1)")
    ap.add_argument("--no-gpu-probe", action="store_true")
    ap.add_argument("--probe-kb", type=int, default=-1,
                    help="HTTP GET probe size in KiB, the rest as parallel Range streams "
                         "(-1: worker default, 0: open-ended probe)")
    ap.add_argument("--http-segments", type=int, default=0, help="max parallel Range streams (0: worker default)")
    ap.add_argument("--sign-threads", type=int, default=0, help="S3 chunk hashers per PUT (0: worker default)")
    ap.add_argument("--log-level", default="warning")
    a = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    cuda = torch.cuda.is_available()
    if cuda:
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    if world > 1:
        dist.init_process_group("nccl" if cuda else "gloo")

    def barrier() -> None:
        if world > 1:
            dist.barrier()
        if cuda:
            torch.cuda.synchronize()

    from tritondl.bench_job import JobStack
    from tritondl.utils.log import log
    log.configure(a.log_level, "")

    file_size = int(a.file_mb * 1024 * 1024)
    stack = JobStack(file_size=file_size, concurrency=a.concurrency, prefetch=max(1, a.concurrency),
                     tag=f"r{rank}", http_probe_bytes=(a.probe_kb << 10) if a.probe_kb >= 0 else -1,
                     http_segments=a.http_segments, sign_threads=a.sign_threads)
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    try:
        loop.run_until_complete(stack.setup())
        c = stack.cfg
        knobs = {"http_probe_bytes": c.http_probe_bytes, "http_segments": c.http_segments,
                 "s3_sign_threads": c.s3_sign_threads} if c is not None else {}
        if a.warmup:
            loop.run_until_complete(stack.run_jobs(a.warmup))
        barrier()
        t0 = time.perf_counter()
        loop.run_until_complete(stack.run_jobs(a.steps))
        if cuda:
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        barrier()
        done = stack.svc.results[-a.steps:]  # type: ignore[union-attr]
        lat = sorted(r.seconds for r in done)
        spans: dict[str, list[float]] = {}
        for r in done:
            for k, v in r.marks.items():
                spans.setdefault(k, []).append(v)
    finally:
        loop.run_until_complete(stack.teardown())
        loop.close()

    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if cuda and world > 1 else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    max_elapsed = float(t.item())
    extra = {} if (a.no_gpu_probe or rank != 0) else _gpu_hash_probe()
    if rank == 0:
        jobs_per_sec = world * a.steps / max_elapsed
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
            "data": f"synthetic (deterministic pseudo-random {file_size / 2**20:g} MiB payload; "
                    "local fake broker/origin/S3)",
            "config": {"model": CONFIG_NAME if file_size == 10 << 20 else
                       f"Single HTTP download job via local RabbitMQ, {file_size / 2**20:g} MiB file", "global_batch": world * a.concurrency, "seq_len": None,
                       "file_bytes": file_size, "parallelism": f"dp{world}",
                       "concurrency_per_worker": a.concurrency, "prefetch": max(1, a.concurrency),
                       **knobs},
            "ingest_MB_per_sec": round(jobs_per_sec * file_size / 1e6, 1),
            "job_latency_ms_p50": round(lat[len(lat) // 2] * 1000, 2) if lat else None,
            "job_latency_ms_p90": round(lat[int(len(lat) * 0.9)] * 1000, 2) if lat else None,
            # median ms from taking the job to the end of each stage (rank 0)
            "job_spans_ms_p50": {k: round(sorted(v)[len(v) // 2] * 1000, 2) for k, v in spans.items()},
        }
        res.update(extra)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
