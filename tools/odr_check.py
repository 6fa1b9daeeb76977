#!/usr/bin/env python3
"""Link-time ODR check for the shared native headers (``csrc/**/*.h``).

Each extension is one translation unit, so a non-``inline`` function or
variable defined in a header links fine today and breaks the day a second
TU includes it.  This compiles ``csrc/tests/odr_tu.cpp`` (which includes
every shared header) twice, as two TUs, and links them into one program:
any header definition that is not ``inline`` / ``static`` / a template is a
"multiple definition" error.  Run by CI (``make odr-check``) and by
``tests/test_tooling.py``.
"""

from __future__ import annotations

import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "tests", "odr_tu.cpp")


def main() -> int:
    with tempfile.TemporaryDirectory() as d:
        objs = []
        for tu in (1, 2):
            o = os.path.join(d, f"tu{tu}.o")
            r = subprocess.run(["g++", "-std=c++17", "-O0", "-w", "-c", f"-DODR_TU={tu}", SRC, "-o", o],
                               capture_output=True, text=True)
            if r.returncode:
                print(r.stderr, file=sys.stderr)
                return r.returncode
            objs.append(o)
        r = subprocess.run(["g++", *objs, "-o", os.path.join(d, "odr"), "-lssl", "-lcrypto", "-pthread"],
                           capture_output=True, text=True)
        if r.returncode:
            dups = sorted({ln.split("multiple definition of", 1)[1].strip()
                           for ln in r.stderr.splitlines() if "multiple definition of" in ln})
            print("ODR check FAILED: header definitions that are not inline:", file=sys.stderr)
            for x in dups or [r.stderr]:
                print("  " + x, file=sys.stderr)
            return 1
    print("ODR check OK: every shared header links into two TUs")
    return 0


if __name__ == "__main__":
    sys.exit(main())
