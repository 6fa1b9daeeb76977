#!/usr/bin/env python3
"""Build and run csrc/tests/native_selftest.cpp (host C++ cores: hashing,
aws-chunked signing, threaded piece verification, the relay pumps, uTP engine,
the BitTorrent peer-wire parser with seeded fuzzing).

    python tools/native_selftest.py              # plain -O2 build
    python tools/native_selftest.py --sanitize   # ASan+UBSan build, then TSan build

Host code only: GPU sanitizers are not used on this pool.
"""

from __future__ import annotations

import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "tests", "native_selftest.cpp")


def build_and_run(flags: list[str], label: str, quick: bool) -> int:
    out = os.path.join(tempfile.gettempdir(), f"tritondl_selftest_{label}")
    cmd = ["g++", "-std=c++17", "-g", *flags, SRC, "-o", out, "-lssl", "-lcrypto", "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        print(r.stdout, r.stderr, file=sys.stderr)
        return r.returncode
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([out] + (["--quick"] if quick else []), env=env, capture_output=True, text=True)
    print(f"[{label}] rc={r.returncode} {r.stdout.strip()} {r.stderr.strip()[-2000:]}")
    return r.returncode


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sanitize", action="store_true")
    a = ap.parse_args()
    if not a.sanitize:
        return build_and_run(["-O2", "-Wall", "-Wextra"], "plain", quick=False)
    rc = build_and_run(["-O1", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=undefined"], "asan_ubsan", quick=True)
    rc |= build_and_run(["-O1", "-fsanitize=thread"], "tsan", quick=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
