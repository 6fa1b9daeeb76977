#!/usr/bin/env python3
"""Build and run csrc/tests/cost_probe.cpp: the thread-CPU floor of each
primitive of a 10 MiB headline job's data path (chunk hashing from a hot
buffer / a fresh mapping / pread scratch, the download's pwrites, loopback
receive, sendfile, unlink).  One JSON line per probe.

    python tools/cost_probe.py [--dir /tmp] [--reps 30]
"""

from __future__ import annotations

import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "tests", "cost_probe.cpp")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=tempfile.gettempdir())
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    out = os.path.join(tempfile.gettempdir(), "tritondl_cost_probe")
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-Wno-deprecated-declarations", SRC, "-o", out, "-lssl", "-lcrypto", "-pthread"],
                       capture_output=True, text=True)
    if r.returncode:
        print(r.stdout, r.stderr, file=sys.stderr)
        return r.returncode
    return subprocess.run([out, "--dir", a.dir, "--reps", str(a.reps)]).returncode


if __name__ == "__main__":
    sys.exit(main())
