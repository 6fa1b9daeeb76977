"""GPU helper churn soak: start → verify → idle exit, many times over.

A long-running worker starts the GPU helper on a torrent resume and lets it
exit after ``TRITONDL_GPU_IDLE_S`` of idleness (``ops/gpu_helper.py``), so
over days it starts and stops HIP hundreds of times.  This runs that cycle
``--cycles`` times with a short idle timeout and reports, per cycle: helper
start + verify latency, its exit status, whether a corrupted piece was
caught, and the driving process's RSS / fds / threads; plus the card's VRAM
in use after each exit when sysfs shows exactly one card.  Anything the
helper leaks on the card or in the worker shows up as drift.

    python tools/gpu_churn.py --cycles 100 --mb 256 --out gpurun_out/churn.jsonl
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _vram_used() -> int | None:
    """VRAM in use on the card, when sysfs shows exactly one; with several
    cards (other tenants' included) the sum would not be this process's."""
    cards = glob.glob("/sys/class/drm/card*/device/mem_info_vram_used")
    if len(cards) != 1:
        return None
    try:
        with open(cards[0]) as fh:
            return int(fh.read())
    except (OSError, ValueError):
        return None


def _proc() -> dict:
    out = {"fds": len(os.listdir("/proc/self/fd")), "threads": len(os.listdir("/proc/self/task"))}
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                out["rss_mb"] = round(int(line.split()[1]) / 1024, 1)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=100)
    ap.add_argument("--mb", type=int, default=256, help="file verified per cycle")
    ap.add_argument("--piece-kb", type=int, default=1024)
    ap.add_argument("--idle", type=float, default=0.5, help="helper idle timeout (s)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    os.environ["TRITONDL_GPU_IDLE_S"] = str(a.idle)
    from tritondl.ops import hashing
    from tritondl.ops.gpu_helper import GpuHelper

    plen = a.piece_kb << 10
    data = os.urandom(a.mb << 20)
    expected = hashing.piece_hashes(data, plen, "sha1")
    npieces = len(expected) // 20
    fd, path = tempfile.mkstemp(prefix="tritondl-churn-", dir=os.environ.get("TMPDIR", "/tmp"))
    with os.fdopen(fd, "wb") as f:
        f.write(data)
    del data
    sink = open(a.out, "w") if a.out else None
    h = GpuHelper(start_timeout=120, call_timeout=120)
    rows = []
    vram0 = _vram_used()
    base = _proc()
    bad_exits = missed = 0
    try:
        for i in range(a.cycles):
            exp = bytearray(expected)
            corrupt = i % 5 == 4                       # every fifth cycle: one piece must fail
            victim = (i * 7919) % npieces
            if corrupt:
                exp[20 * victim] ^= 0xFF
            t0 = time.perf_counter()
            ok = h.verify_files([(path, os.path.getsize(path))], plen, bytes(exp), "sha1")
            dt = time.perf_counter() - t0
            want_bad = {victim} if corrupt else set()
            got_bad = {k for k in range(npieces) if not ok[k]}
            if got_bad != want_bad:
                missed += 1
            pid = h.pid
            exited = h.wait_exit(a.idle + 30)
            rc = h._p.returncode if h._p is not None else None
            if not exited or rc != 0:
                bad_exits += 1
            row = {"cycle": i, "helper_pid": pid, "start_verify_s": round(dt, 3), "gpu_pieces": h.last_gpu_pieces,
                   "exit_rc": rc, "exited": exited, "bad_pieces_ok": got_bad == want_bad,
                   "vram_used_mb": (None if (v := _vram_used()) is None else round(v / 2**20, 1)), **_proc()}
            rows.append(row)
            line = json.dumps(row)
            print(line, flush=True)
            if sink:
                sink.write(line + "\n")
                sink.flush()
    finally:
        h.close()
        os.unlink(path)
    lat = sorted(r["start_verify_s"] for r in rows)
    half = len(rows) // 2
    summary = {
        "cycles": len(rows), "spawned": h.spawned, "mb_per_cycle": a.mb, "pieces": npieces,
        "verify_mismatches": missed, "bad_exits": bad_exits,
        "start_verify_s": {"p50": lat[len(lat) // 2], "p99": lat[min(len(lat) - 1, int(len(lat) * 0.99))],
                           "max": lat[-1]} if lat else None,
        "gpu_pieces_min": min((r["gpu_pieces"] for r in rows), default=None),
        "rss_mb": [base.get("rss_mb"), rows[-1]["rss_mb"]] if rows else None,
        "fds": [base["fds"], rows[-1]["fds"]] if rows else None,
        "threads": [base["threads"], rows[-1]["threads"]] if rows else None,
        "vram_used_mb_first_half_max": max((r["vram_used_mb"] or 0 for r in rows[:half]), default=None),
        "vram_used_mb_second_half_max": max((r["vram_used_mb"] or 0 for r in rows[half:]), default=None),
        "vram_used_mb_before": None if vram0 is None else round(vram0 / 2**20, 1),
    }
    print(json.dumps({"summary": summary}), flush=True)
    if sink:
        sink.write(json.dumps({"summary": summary}) + "\n")
        sink.close()
    return 0 if not missed and not bad_exits and h.spawned == len(rows) else 1


if __name__ == "__main__":
    sys.exit(main())
