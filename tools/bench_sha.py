#!/usr/bin/env python3
"""SHA-256 throughput of the aws-chunked hot loop: OpenSSL vs the two-stream
SHA-NI path (csrc/hash/sha_ni.h).

Runs ``hashing.chunk_signatures`` over a buffer of 64 KiB chunks on 1 and
N threads in two child processes, one with ``TRITONDL_SHA_NI=0`` (OpenSSL
for every digest) and one with the default setting.  The switch is read
once per process, so each setting needs its own child.  Prints one JSON
line per (mode, threads).

    python tools/bench_sha.py [--mb 256] [--threads 1,4,8]
"""

from __future__ import annotations

import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
sys.path.insert(0, {root!r})
from tritondl.ops import hashing
data = os.urandom({mb} << 20)
key = b"k" * 32
for t in {threads}:
    hashing.chunk_signatures(key, "20240101T000000Z", "s", "0" * 64, data[:1 << 20], 65536, threads=t)   # warm
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        hashing.chunk_signatures(key, "20240101T000000Z", "s", "0" * 64, data, 65536, threads=t)
        best = min(best, time.perf_counter() - t0)
    print(json.dumps({{"mode": {mode!r}, "threads": t, "MB_per_sec": round(len(data) / best / 1e6, 1)}}), flush=True)
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=256)
    ap.add_argument("--threads", default="1,4,8")
    a = ap.parse_args()
    threads = [int(x) for x in a.threads.split(",")]
    rc = 0
    for mode, env in (("openssl", "0"), ("sha_ni_x2", "1")):
        code = CHILD.format(root=ROOT, mb=a.mb, threads=threads, mode=mode)
        r = subprocess.run([sys.executable, "-c", code], env={**os.environ, "TRITONDL_SHA_NI": env})
        rc |= r.returncode
    return rc


if __name__ == "__main__":
    sys.exit(main())
