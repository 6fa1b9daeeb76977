#!/usr/bin/env python3
"""Where does GPU resume-verification time go?  Host->HBM staging probe.

The HIP verify pipeline is: file bytes (page cache) --pread--> pinned staging
--hipMemcpyAsync (SDMA, PCIe)--> HBM window --kernel--> digests.  This tool
times each hop on its own, on the same files, so the pipeline's ceiling can
be attributed (SURVEY §5.4 resume; VERDICT r1 "lift the ~45 GB/s staging
ceiling"):

  1. buffered pread into pinned memory, T threads (page cache hot)
  2. O_DIRECT pread into page-aligned memory, T threads (bypasses the cache:
     what a cache-cold resume would see; EINVAL on filesystems without it)
  3. pinned -> HBM copies, 1 and 2 HIP streams (two SDMA queues)
  4. the production verifiers on the whole layout: host (SHA-NI threads),
     GPU with R reader threads, hybrid (GPU + CPU threads from the other end)

    python tools/staging_probe.py --gb 8 [--files 4] [--piece-kb 1024]

One JSON line per measurement.
"""

from __future__ import annotations

import argparse
import json
import mmap
import os
import shutil
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def emit(**kw) -> None:
    print(json.dumps(kw), flush=True)


def parallel_pread(paths: list[str], buf: memoryview, threads: int, flags: int = 0, unit: int = 8 << 20) -> float:
    """Read every file back to back into buf with `threads` threads; GB/s."""
    sizes = [os.path.getsize(p) for p in paths]
    jobs = []
    off = 0
    for p, n in zip(paths, sizes):
        for a in range(0, n, unit):
            jobs.append((p, a, min(unit, n - a), off + a))
        off += n
    fds = {p: os.open(p, os.O_RDONLY | flags) for p in paths}
    lock = threading.Lock()
    it = iter(jobs)
    err: list[BaseException] = []

    def work() -> None:
        while True:
            with lock:
                j = next(it, None)
            if j is None:
                return
            p, a, n, dst = j
            try:
                got = os.preadv(fds[p], [buf[dst:dst + n]], a)
                if got != n:
                    raise OSError(f"short read {got}/{n}")
            except OSError as e:
                err.append(e)
                return

    t0 = time.perf_counter()
    ts = [threading.Thread(target=work) for _ in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    for fd in fds.values():
        os.close(fd)
    if err:
        raise err[0]
    return off / dt / 1e9


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=8.0)
    ap.add_argument("--files", type=int, default=4)
    ap.add_argument("--piece-kb", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    import torch

    from tritondl.ops import hashing

    td = tempfile.mkdtemp(prefix="tdl-stage-", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        total = int(a.gb * (1 << 30)) // a.files * a.files
        per = total // a.files
        paths = []
        rng = np.random.default_rng(7)
        block = rng.integers(0, 256, 64 << 20, dtype=np.uint8).tobytes()
        for k in range(a.files):
            p = os.path.join(td, f"e{k}.bin")
            with open(p, "wb") as f:
                left = per
                while left:
                    n = min(left, len(block))
                    f.write(block[:n] if k == 0 else bytes(np.roll(np.frombuffer(block[:n], np.uint8), k)))
                    left -= n
            paths.append(p)
        emit(probe="setup", bytes=total, files=a.files, cpus=hashing.effective_cpus())
        # 1. buffered pread -> pinned (what the GPU readers do)
        pinned = torch.empty(total, dtype=torch.uint8, pin_memory=True)
        pmv = memoryview(pinned.numpy()).cast("B")
        for thr in (4, 8, 12, 16):
            best = max(parallel_pread(paths, pmv, thr) for _ in range(a.reps))
            emit(probe="pread_buffered_to_pinned", threads=thr, GBps=round(best, 1))
        # 2. O_DIRECT (page-aligned anonymous memory)
        am = mmap.mmap(-1, total)
        amv = memoryview(am)
        for thr in (8, 16):
            try:
                g = parallel_pread(paths, amv, thr, flags=getattr(os, "O_DIRECT", 0))
                emit(probe="pread_odirect", threads=thr, GBps=round(g, 1))
            except OSError as e:
                emit(probe="pread_odirect", threads=thr, error=str(e))
                break
        amv.release()
        am.close()
        # 3. pinned -> HBM
        dev = torch.device("cuda:0")
        chunk = 1 << 30
        dbuf = torch.empty(total, dtype=torch.uint8, device=dev)
        for nstreams in (1, 2, 4):
            streams = [torch.cuda.Stream() for _ in range(nstreams)]
            best = 0.0
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i, off in enumerate(range(0, total, chunk)):
                    n = min(chunk, total - off)
                    with torch.cuda.stream(streams[i % nstreams]):
                        dbuf[off:off + n].copy_(pinned[off:off + n], non_blocking=True)
                torch.cuda.synchronize()
                best = max(best, total / (time.perf_counter() - t0) / 1e9)
            emit(probe="h2d_pinned_to_hbm", streams=nstreams, GBps=round(best, 1))
        del dbuf, pinned
        torch.cuda.empty_cache()
        # 4. production verifiers over the layout
        piece = a.piece_kb << 10
        files = [(p, per) for p in paths]
        blob_hash = hashing.verify_pieces  # noqa: F841 - keep the import explicit
        exp = b"".join(hashing._host.piece_hashes("sha1", open(p, "rb").read(), piece, hashing.effective_cpus())
                       for p in paths) if per % piece == 0 else None
        if exp is None:
            emit(probe="verify", error="file size must be a multiple of the piece size")
            return 1
        n = total // piece
        for dev_name, env in (("cpu", {}), ("gpu", {"TRITONDL_GPU_READERS": "8"}),
                              ("gpu", {"TRITONDL_GPU_READERS": "12"}), ("gpu", {"TRITONDL_GPU_READERS": "16"}),
                              ("hybrid", {"TRITONDL_GPU_READERS": "8", "TRITONDL_HYBRID_CPU_THREADS": "8"}),
                              ("hybrid", {"TRITONDL_GPU_READERS": "8", "TRITONDL_HYBRID_CPU_THREADS": "4"}),
                              ("hybrid", {"TRITONDL_GPU_READERS": "12", "TRITONDL_HYBRID_CPU_THREADS": "6"}),
                              ("hybrid", {"TRITONDL_GPU_READERS": "6", "TRITONDL_HYBRID_CPU_THREADS": "10"})):
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                times = []
                for _ in range(a.reps + 1):          # first GPU run pays set-up
                    t0 = time.perf_counter()
                    ok = hashing.verify_pieces(files, piece, exp, device=dev_name)
                    times.append(time.perf_counter() - t0)
                    assert sum(ok) == n
                best = min(times[1:])
                extra = {}
                if dev_name == "hybrid":
                    extra["gpu_share"] = round(hashing.gpu_hasher().last_gpu_pieces / n, 3)
                emit(probe="verify", device=dev_name, **env, seconds=round(best, 3),
                     GBps=round(total / best / 1e9, 1), **extra)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
    finally:
        shutil.rmtree(td, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
