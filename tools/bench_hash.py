#!/usr/bin/env python3
"""Micro-benchmark of the piece-hash paths (one JSON line per case).

* gpu_kernel   : HIP kernel on device-resident data (hash_device), GB/s
* gpu_pipeline : GpuHasher.hash_buffer from host memory (H2D + kernel + D2H)
* gpu_verify   : GpuHasher.verify_files over files in the page cache
* cpu_pieces   : host OpenSSL piece_hashes, all threads
* cpu_verify   : host verify_pieces over the same files
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--total-mb", type=int, default=1024)
    ap.add_argument("--piece-kb", type=int, nargs="*", default=[16, 256, 1024, 4096])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kinds", nargs="*", default=["sha1", "sha256"])
    ap.add_argument("--no-files", action="store_true")
    ap.add_argument("--lanes", type=int, nargs="*", default=[64], help="pieces per wavefront (16/32/64)")
    ap.add_argument("--kernel-only", action="store_true")
    a = ap.parse_args()

    import numpy as np

    from tritondl.ops import hashing

    total = a.total_mb << 20
    host = np.random.default_rng(0).integers(0, 256, total, dtype=np.uint8)
    have_gpu = hashing.gpu_available()
    res = []
    if have_gpu:
        import torch
        dev = torch.from_numpy(host).cuda()
        stream = torch.cuda.current_stream().cuda_stream
        mod = hashing.gpu_module()
    for kind in a.kinds:
        dl = 20 if kind == "sha1" else 32
        for pk in a.piece_kb:
            pl = pk << 10
            n = (total + pl - 1) // pl
            if have_gpu:
                out = torch.empty(n * dl, dtype=torch.uint8, device="cuda")
                for lanes in a.lanes:
                    def k():
                        mod.hash_device(kind, dev.data_ptr(), total, pl, out.data_ptr(), stream, lanes)
                        torch.cuda.synchronize()
                    t = timeit(k, a.reps)
                    res.append({"case": "gpu_kernel", "kind": kind, "piece_kb": pk, "pieces": n, "lanes": lanes,
                                "GBps": total / t / 1e9, "ms": t * 1e3})
                    print(json.dumps(res[-1]), flush=True)
                if a.kernel_only:
                    continue
                t = timeit(lambda: hashing.piece_hashes(host, pl, kind, device="gpu"), max(1, a.reps // 2))
                res.append({"case": "gpu_pipeline", "kind": kind, "piece_kb": pk, "GBps": total / t / 1e9,
                            "ms": t * 1e3})
            t = timeit(lambda: hashing.piece_hashes(host, pl, kind, device="cpu"), max(1, a.reps // 2))
            res.append({"case": "cpu_pieces", "kind": kind, "piece_kb": pk, "threads": os.cpu_count(),
                        "GBps": total / t / 1e9, "ms": t * 1e3})
            for r in res[-2:]:
                print(json.dumps(r), flush=True)
    if not a.no_files:
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
            files = []
            per = total // 4
            for i in range(4):
                p = os.path.join(td, f"f{i}")
                host[i * per:(i + 1) * per].tofile(p)
                files.append((p, per))
            pl = 1 << 20
            exp = hashing.piece_hashes(host[:per * 4], pl, "sha1", device="cpu")
            t = timeit(lambda: hashing.verify_pieces(files, pl, exp, device="cpu"), 2)
            r = {"case": "cpu_verify", "piece_kb": 1024, "GBps": per * 4 / t / 1e9, "ms": t * 1e3}
            print(json.dumps(r), flush=True)
            if have_gpu:
                ok = hashing.verify_pieces(files, pl, exp, device="gpu")
                assert all(ok), "gpu verify mismatch"
                t = timeit(lambda: hashing.verify_pieces(files, pl, exp, device="gpu"), 2)
                r = {"case": "gpu_verify", "piece_kb": 1024, "GBps": per * 4 / t / 1e9, "ms": t * 1e3}
                print(json.dumps(r), flush=True)
            # BitTorrent v2 (BEP 52): per-piece merkle roots over 16 KiB leaves
            from tritondl.fetch.bt.metainfo import make_info
            info = make_info(td, 1 << 20, version=2)
            layout = info.file_paths(os.path.dirname(td))
            exp2, widths, reals, known = info.v2_expectations()
            nbytes = info.total_length
            cpu = hashing.verify_pieces_v2(layout, info.piece_length, exp2, widths, reals, known, device="cpu")
            assert all(cpu), "cpu v2 verify mismatch"
            t = timeit(lambda: hashing.verify_pieces_v2(layout, info.piece_length, exp2, widths, reals, known,
                                                        device="cpu"), 2)
            print(json.dumps({"case": "cpu_verify_v2", "piece_kb": 1024, "GBps": nbytes / t / 1e9, "ms": t * 1e3,
                              "threads": hashing.effective_cpus()}), flush=True)
            if have_gpu:
                ok = hashing.verify_pieces_v2(layout, info.piece_length, exp2, widths, reals, known, device="gpu")
                assert ok == cpu, "gpu v2 verify mismatch"
                t = timeit(lambda: hashing.verify_pieces_v2(layout, info.piece_length, exp2, widths, reals, known,
                                                            device="gpu"), 2)
                print(json.dumps({"case": "gpu_verify_v2", "piece_kb": 1024, "GBps": nbytes / t / 1e9,
                                  "ms": t * 1e3}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
