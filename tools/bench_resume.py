#!/usr/bin/env python3
"""Resume benchmark: a redelivered torrent job whose data is already on disk
(the worker crashed after downloading, before the ack — SURVEY.md §5.4).
The production ``TorrentDownloader`` opens the job from a ``.torrent``,
batch-verifies the existing files and completes with nothing left to fetch;
the job time is almost entirely verification, so this is where the HIP
kernels sit on the service path.

    python tools/bench_resume.py --gb 4 --version 2 --device gpu|cpu|auto
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
    ap.add_argument("--gb", type=float, default=4.0)
    ap.add_argument("--files", type=int, default=4)
    ap.add_argument("--piece-kb", type=int, default=1024)
    ap.add_argument("--version", type=int, default=2, choices=[1, 2, 3])
    ap.add_argument("--device", nargs="*", default=["cpu", "gpu"])
    ap.add_argument("--reps", type=int, default=2, help="runs per device; the first GPU run pays HIP set-up")
    ap.add_argument("--trace", action="store_true", help="GPU event timeline summary per run")
    ap.add_argument("--cpus", default="", help="pin the run (file writes, so page-cache placement, and hashing "
                                               "threads) to this cpulist")
    a = ap.parse_args()
    if a.cpus:
        from tritondl.parallel.topology import parse_cpulist
        os.sched_setaffinity(0, parse_cpulist(a.cpus))
    import numpy as np

    from tritondl_testkit.fakes.origin import Origin
    from tritondl_testkit.fakes.swarm import torrent_file_bytes
    from tritondl.fetch.bt.client import TorrentDownloader
    from tritondl.fetch.bt.metainfo import make_info
    from tritondl.fetch.bt.torrent import TorrentConfig
    from tritondl.ops import hashing
    from tritondl.utils.log import log
    log.configure("warning", "")
    td = tempfile.mkdtemp(prefix="tdl-resume-", dir=os.environ.get("TMPDIR", "/tmp"))
    o = None
    try:
        root = os.path.join(td, "job", "Season")
        os.makedirs(root)
        total = int(a.gb * (1 << 30))
        per = total // a.files
        rng = np.random.default_rng(3)
        for k in range(a.files):
            rng.integers(0, 256, per, dtype=np.uint8).tofile(os.path.join(root, f"e{k:02d}.mkv"))
        t0 = time.perf_counter()
        info = make_info(root, a.piece_kb << 10, version=a.version)
        t_make = time.perf_counter() - t0
        o = await Origin().start()
        url = o.add("/job.torrent", torrent_file_bytes(info))
        spent = {"verify_s": 0.0}
        for name in ("verify_pieces", "verify_pieces_v2"):
            real = getattr(hashing, name)

            def timed(*args, _real=real, **kw):
                t = time.perf_counter()
                try:
                    return _real(*args, **kw)
                finally:
                    spent["verify_s"] += time.perf_counter() - t
            setattr(hashing, name, timed)
        for dev in a.device:
            if dev in ("gpu", "hybrid") and not hashing.gpu_available():
                continue
            for rep in range(a.reps):
                # the same files, but no completion DB: the job must re-verify everything
                db = os.path.join(td, "job", ".torrent.db")
                for suffix in ("", "-wal", "-shm"):
                    if os.path.exists(db + suffix):
                        os.remove(db + suffix)
                if a.trace and dev in ("gpu", "hybrid") and not hashing.helper_mode():
                    hashing.gpu_hasher().trace = True
                d = TorrentDownloader(TorrentConfig(listen_host="127.0.0.1", verify_device=dev), use_dht=False,
                                      progress_interval=1.0)
                spent["verify_s"] = 0.0
                t0 = time.perf_counter()
                await d.download(os.path.join(td, "job"), lambda u, p: None, url)
                dt = time.perf_counter() - t0
                extra = {"verify_s": round(spent["verify_s"], 3)}
                if dev in ("gpu", "hybrid", "auto") and hashing.gpu_available():
                    h = hashing.gpu_backend()           # the helper process's hasher by default
                    if dev != "gpu":
                        extra["gpu_share"] = round(h.last_gpu_pieces / max(1, info.num_pieces if info.pieces
                                                                            else -(-info.total_length // 16384)), 3)
                    extra["direct_share"] = round(h.last_direct_bytes / max(1, info.total_length), 3)
                    if getattr(h, "trace", False):
                        extra["gpu_timeline"] = hashing.timeline_summary(h.last_timeline)
                print(json.dumps({"metric": "resume_job_seconds", "device": dev, "run": "cold" if rep == 0 else "warm",
                                  "value": round(dt, 3), "GBps": round(info.total_length / dt / 1e9, 1),
                                  "bytes": info.total_length, "pieces": info.num_pieces,
                                  "torrent_version": a.version, "make_torrent_s": round(t_make, 2), **extra}),
                      flush=True)
    finally:
        if o is not None:
            await o.stop()
        shutil.rmtree(td, ignore_errors=True)
    if a.cpus and any(d != "cpu" for d in a.device):
        from tritondl.parallel.topology import gpu_numa_node
        print(json.dumps({"cpus": a.cpus, "gpu_numa_node": gpu_numa_node(0)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(asyncio.run(main()))
