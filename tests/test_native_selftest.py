"""Builds and runs the standalone C++ self-test of the host native cores
(hash_core.h, utp_engine.h) — the same binary CI runs under ASan/UBSan/TSan."""

import subprocess
import sys

from .conftest import ROOT


def test_native_selftest_plain_build():
    r = subprocess.run([sys.executable, "tools/native_selftest.py"], cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "native selftest OK" in r.stdout
