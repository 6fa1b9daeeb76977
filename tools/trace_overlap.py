#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace --memory-copy-trace`` CSV run:
how long the GPU spent in kernels, in host<->device copies, and how much of
the two overlapped (the HIP verify pipeline copies window k+1 on one stream
while window k hashes on another).

    python tools/trace_overlap.py gpurun_out/prof/resume_trace   # dir holding *_kernel_trace.csv etc.

Prints one JSON object.
"""

from __future__ import annotations

import csv
import glob
import json
import os
import sys


def _rows(pattern: str) -> list[dict]:
    out: list[dict] = []
    for p in glob.glob(pattern, recursive=True):
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def _col(row: dict, *keys: str) -> str | None:
    low = {k.lower(): k for k in row}
    for k in keys:
        if k.lower() in low:
            return low[k.lower()]
    return None


def _intervals(rows: list[dict]) -> list[tuple[int, int]]:
    if not rows:
        return []
    s = _col(rows[0], "Start_Timestamp", "start_timestamp", "BeginNs", "Start")
    e = _col(rows[0], "End_Timestamp", "end_timestamp", "EndNs", "End")
    if s is None or e is None:
        raise SystemExit(f"no start/end columns in {list(rows[0])}")
    return sorted((int(r[s]), int(r[e])) for r in rows if r.get(s) and r.get(e))


def _union(iv: list[tuple[int, int]]) -> list[tuple[int, int]]:
    out: list[list[int]] = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return [(a, b) for a, b in out]


def _length(iv: list[tuple[int, int]]) -> int:
    return sum(b - a for a, b in iv)


def _intersect(x: list[tuple[int, int]], y: list[tuple[int, int]]) -> int:
    i = j = tot = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main() -> int:
    d = sys.argv[1] if len(sys.argv) > 1 else "."
    kern = _rows(os.path.join(d, "**", "*kernel_trace.csv"))
    copy = _rows(os.path.join(d, "**", "*memory_copy_trace.csv"))
    hash_k = [r for r in kern if "hash_pieces" in r.get(_col(r, "Kernel_Name", "KernelName") or "", "")]
    ki = _union(_intervals(hash_k))
    res: dict = {"hash_kernels": len(hash_k), "copies": len(copy)}
    res["kernel_busy_ms"] = round(_length(ki) / 1e6, 3)
    if copy:
        dcol = _col(copy[0], "Direction", "Kind", "Operation")
        bcol = _col(copy[0], "Bytes", "Size", "Copy_Bytes")
        h2d = [r for r in copy if dcol is None or "HOST_TO_DEVICE" in r[dcol].upper() or "H2D" in r[dcol].upper()]
        ci = _union(_intervals(h2d))
        res["h2d_copies"] = len(h2d)
        res["h2d_busy_ms"] = round(_length(ci) / 1e6, 3)
        if bcol is not None:
            nbytes = sum(int(r[bcol] or 0) for r in h2d)
            res["h2d_bytes"] = nbytes
            if ci:
                res["h2d_GBps_while_busy"] = round(nbytes / max(1, _length(ci)), 2)
        res["kernel_overlapped_by_h2d_ms"] = round(_intersect(ki, ci) / 1e6, 3)
        all_iv = _union(ki + ci)
        if all_iv:
            res["span_ms"] = round((all_iv[-1][1] - all_iv[0][0]) / 1e6, 3)
            res["gpu_busy_ms"] = round(_length(all_iv) / 1e6, 3)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
