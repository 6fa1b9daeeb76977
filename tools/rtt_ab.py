#!/usr/bin/env python3
"""Worker defaults under realistic round trips.

Loopback fakes answer in ~0.05 ms, so every earlier A/B of a latency knob
measured nothing: broker confirms, S3 responses and origin TTFB cost 1-50 ms
in production.  This runs ``bench.py`` with the fakes' emulated network
(``--rtt-ms``: one RTT per new connection, TLS handshake, request/response
and broker frame; ``--stream-mbps``: one stream's window/RTT throughput cap)
over the knobs chosen on loopback, and writes one JSON line per run plus a
markdown table.

    python tools/rtt_ab.py --out gpurun_out/r05_rtt_ab [--rtts 2,20] [--quick]

Every run is a separate ``bench.py`` process under its own time limit.
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (name, bench args, what it tests)
SMALL = [
    ("default", ["--pipeline-commit", "off"], "round-4 defaults (concurrency 1, prefetch 1, pipeline_commit off)"),
    ("pipeline_commit", ["--pipeline-commit", "on"], "publish confirm + ack overlap the next job (prefetch 1)"),
    ("pipeline_commit+prefetch2", ["--pipeline-commit", "on", "--prefetch", "2"],
     "pipelined commit with room on the shard for the next delivery"),
    ("probe_1MiB", ["--probe-kb", "1024"], "bounded GET probe, the rest as parallel Range streams"),
    ("segments_1", ["--http-segments", "1"], "one stream per file"),
    ("concurrency_2", ["--concurrency", "2"], "two jobs in flight (prefetch 2)"),
    ("concurrency_4", ["--concurrency", "4"], "four jobs in flight (prefetch 4)"),
]
# a 256 MiB job with each stream capped (window / RTT): what segments and multipart are for
BIG = [
    ("big_default", [], "256 MiB: defaults (4 Range streams >= 64 MiB; multipart 16 MiB x 4 parallel)"),
    ("big_segments_1", ["--http-segments", "1"], "256 MiB: one download stream"),
    ("big_segments_8", ["--http-segments", "8"], "256 MiB: 8 download streams"),
    ("big_single_put", ["--s3-multipart-mb", "1024"], "256 MiB: one PUT (no multipart)"),
    ("big_parts_64MiB", ["--s3-part-mb", "64"], "256 MiB: 64 MiB parts (4 parts)"),
    ("big_parallel_parts_8", ["--s3-parallel-parts", "8"], "256 MiB: 8 parts in flight"),
    ("big_segments_8_parts_8", ["--http-segments", "8", "--s3-parallel-parts", "8"],
     "256 MiB: 8 download streams and 8 parts in flight"),
]
# a 32 MiB job (between one part and the 64 MiB multipart threshold), each stream capped
MID = [
    ("mid_default", [], "32 MiB: defaults (one PUT below the 64 MiB multipart threshold)"),
    ("mid_multipart_16", ["--s3-multipart-mb", "16"], "32 MiB: multipart from 16 MiB (2 parts in parallel)"),
    ("mid_multipart_16_segments_probe", ["--s3-multipart-mb", "16", "--http-segments", "4", "--probe-kb", "4096"],
     "32 MiB: 2 parts + a 4 MiB probe and parallel Range streams"),
]
# uncapped (loopback bandwidth), 1 GiB: do more streams cost anything when no stream is capped?
UNCAPPED = [
    ("gib_default", [], "1 GiB, no stream cap: defaults"),
    ("gib_segments_8_parts_8", ["--http-segments", "8", "--s3-parallel-parts", "8"], "1 GiB, no stream cap: 8 x 8"),
]


def run(args: list[str], timeout: float) -> dict:
    t0 = time.monotonic()
    try:
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-gpu-probe", "--no-reference-mode",
                            *args], capture_output=True, text=True, timeout=timeout, cwd="/tmp")
    except subprocess.TimeoutExpired:
        return {"error": f"timeout after {timeout:.0f}s"}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode or not lines:
        return {"error": (p.stderr or p.stdout)[-600:], "rc": p.returncode}
    d = json.loads(lines[-1])
    d["_wall_s"] = round(time.monotonic() - t0, 1)
    return d


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/rtt_ab")
    ap.add_argument("--rtts", default="0,2,20")
    ap.add_argument("--stream-mbps", type=float, default=800.0, help="per-stream cap of the 256 MiB runs")
    ap.add_argument("--quick", action="store_true", help="fewer steps (a smoke run of the matrix)")
    ap.add_argument("--only", default="", help="comma-separated run names")
    ap.add_argument("--repeat", type=int, default=1, help="alternate the selected runs this many times")
    ap.add_argument("--sets", default="small,big", help="small,big,mid,uncapped")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    only = set(filter(None, a.only.split(",")))
    rows = []
    jl = open(os.path.join(a.out, "runs.jsonl"), "a")
    sets = set(a.sets.split(","))

    def one(rtt: float, name: str, what: str, args: list[str], timeout: float) -> None:
        d = run(args, timeout)
        rows.append((rtt, name, what, d))
        jl.write(json.dumps({"rtt_ms": rtt, "name": name, "args": args, "result": d}) + "\n")
        jl.flush()
        print(f"[{time.strftime('%T')}] rtt={rtt} {name}: {d.get('value', d.get('error'))}", flush=True)

    for _rep in range(a.repeat):
        for rtt in [float(x) for x in a.rtts.split(",")]:
            small_steps = 10 if a.quick else (200 if rtt <= 2 else 60)
            cap = ["--stream-mbps", str(a.stream_mbps)]
            plan = []
            if "small" in sets:
                plan += [(n, ["--steps", str(small_steps), "--warmup", "5", *x], w, 240) for n, x, w in SMALL]
            if "mid" in sets:
                plan += [(n, [*cap, "--file-mb", "32", "--steps", "5" if a.quick else "20", "--warmup", "2", *x], w, 240)
                         for n, x, w in MID]
            if "big" in sets:
                plan += [(n, [*cap, "--file-mb", "256", "--steps", "3" if a.quick else "8", "--warmup", "1", *x], w, 300)
                         for n, x, w in BIG]
            if "uncapped" in sets and rtt == 0:
                plan += [(n, ["--file-mb", "1024", "--steps", "3" if a.quick else "6", "--warmup", "1", *x], w, 300)
                         for n, x, w in UNCAPPED]
            for name, extra, what, lim in plan:
                if only and name not in only:
                    continue
                one(rtt, name, what, ["--rtt-ms", str(rtt), *extra], lim)
    jl.close()
    with open(os.path.join(a.out, "TABLE.md"), "w") as f:
        f.write("| RTT ms | run | jobs/s | MB/s | job p50 ms | fetched p50 | upload p50 | ack p50 | what |\n")
        f.write("|---|---|---|---|---|---|---|---|---|\n")
        for rtt, name, what, d in rows:
            if "error" in d:
                f.write(f"| {rtt:g} | {name} | error | | | | | | {what}: {str(d['error'])[:80]} |\n")
                continue
            sp = d.get("job_spans_ms_p50") or {}
            f.write(f"| {rtt:g} | {name} | {d['value']:.1f} | {d['ingest_MB_per_sec']:.0f} | "
                    f"{d.get('job_latency_ms_p50')} | {sp.get('fetched', '')} | {sp.get('upload', '')} | "
                    f"{sp.get('ack', '')} | {what} |\n")
    print(open(os.path.join(a.out, "TABLE.md")).read())
    return 0


if __name__ == "__main__":
    sys.exit(main())
