#!/usr/bin/env python3
"""Development loop (the reference's ``modd.conf``: rebuild + restart on
source change): watch ``tritondl/**/*.py`` and ``csrc/**``; on a change,
rebuild the native extensions if C++/HIP sources changed, then restart the
worker (``python -m tritondl`` with the current environment, e.g. after
``. hack/load-env.sh``).

    python tools/devwatch.py [-- extra worker args]
"""

from __future__ import annotations

import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WATCH = [("tritondl", (".py",)), ("csrc", (".cpp", ".h", ".hip"))]


def snapshot() -> dict[str, float]:
    out = {}
    for d, exts in WATCH:
        for root, _dirs, files in os.walk(os.path.join(ROOT, d)):
            for f in files:
                if f.endswith(exts):
                    p = os.path.join(root, f)
                    try:
                        out[p] = os.path.getmtime(p)
                    except OSError:
                        pass
    return out


def start(args: list[str]) -> subprocess.Popen:
    print("[devwatch] starting worker", flush=True)
    return subprocess.Popen([sys.executable, "-m", "tritondl", *args], cwd=ROOT)


def stop(p: subprocess.Popen) -> None:
    if p.poll() is None:
        p.send_signal(signal.SIGTERM)
        try:
            p.wait(15)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def main() -> int:
    args = sys.argv[sys.argv.index("--") + 1:] if "--" in sys.argv else []
    subprocess.run([sys.executable, "tools/build_native.py"], cwd=ROOT, check=False)
    snap = snapshot()
    proc = start(args)
    try:
        while True:
            time.sleep(1.0)
            cur = snapshot()
            changed = [p for p in cur if cur[p] != snap.get(p)] + [p for p in snap if p not in cur]
            if not changed:
                continue
            snap = cur
            print(f"[devwatch] {len(changed)} file(s) changed: {os.path.relpath(changed[0], ROOT)} ...", flush=True)
            if any(p.startswith(os.path.join(ROOT, "csrc")) for p in changed):
                r = subprocess.run([sys.executable, "tools/build_native.py"], cwd=ROOT)
                if r.returncode:
                    print("[devwatch] native build failed; keeping the old worker", flush=True)
                    continue
            stop(proc)
            proc = start(args)
    except KeyboardInterrupt:
        pass
    finally:
        stop(proc)
    return 0


if __name__ == "__main__":
    sys.exit(main())
