"""A/B: one HTTP/2 connection (``TRITONDL_HTTP2=1``, :mod:`tritondl.fetch.h2`)
against the default HTTP/1.1 path (one TLS connection per Range segment,
bodies read by the native relay) on the same https download.  HTTP/2 runs
three ways: ``h2n``, the relay's TLS with the native session pump
(csrc/relay/h2.h) and up to 4 connections per origin (the default);
``h2n1``, the same on one connection; ``h2``, asyncio's TLS with bodies in
Python, one connection.

Arms, each ``--runs`` times on a fresh origin:

* ``open``   — loopback, no cap: what each client path costs per byte.
* ``stream`` — every response capped at ``--rate`` bytes/s (a CDN's
  per-request pacing): four streams or four connections both get 4x.
* ``conn``   — the h2 connection capped at ``--rate`` (one TCP window over a
  long path), the HTTP/1.1 origin capped per connection the same way:
  HTTP/2's one connection gets 1x where four connections get 4x.

The origin runs in a child process, so ``cpu_s`` is the client's alone.
``python tools/h2_ab.py --out profiles/r06_h2_ab`` writes one JSON line
per run to ``runs.jsonl`` there and prints a table.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tritondl.fetch.http import HTTPDownloader  # noqa: E402
from tritondl.utils import rawhttp  # noqa: E402
from tritondl_testkit.fakes.h2origin import H2Origin  # noqa: E402
from tritondl_testkit.fakes.origin import Origin  # noqa: E402


def _serve(conn, arm: str, proto: str, mib: int, rate: float) -> None:
    """The origin, in a child process: its CPU is not the client's."""
    async def run() -> None:
        data = os.urandom(1 << 20) * mib
        if proto in ("h2", "h2n", "h2n1"):
            o = await H2Origin().start()
            if arm == "stream":
                o.stream_rate = rate
            elif arm == "conn":
                o.conn_rate = rate
            ca = o.ca_pem
        else:
            ca, cert, key = rawhttp.relay_module().make_test_pki(["127.0.0.1"])
            o = await Origin(tls=(cert, key)).start()
            o.rate = rate if arm in ("stream", "conn") else None     # one response per connection: the same cap
        conn.send((o.add("/ab.mkv", data), ca))
        c0 = time.process_time()
        await asyncio.get_running_loop().run_in_executor(None, conn.recv)
        gets = len([r for r in o.requests if r[0] == "GET"])
        conn.send((o.connections if proto in ("h2", "h2n", "h2n1") else gets, time.process_time() - c0))
        await o.stop()
    asyncio.run(run())


async def one(arm: str, proto: str, mib: int, rate: float) -> dict:
    parent, child = mp.Pipe()
    p = mp.get_context("fork").Process(target=_serve, args=(child, arm, proto, mib, rate), daemon=True)
    p.start()
    if not parent.poll(60):
        raise RuntimeError(f"the {proto} origin did not start")
    url, ca = parent.recv()
    d = tempfile.mkdtemp(prefix="tdl-h2ab-")
    if proto in ("h2", "h2n", "h2n1"):
        dl = HTTPDownloader(progress_interval=1.0, ca_pem=ca, http2=True, segment_threshold=16 << 20,
                            h2_native=proto != "h2", h2_conns=4 if proto == "h2n" else 1)
    else:
        dl = HTTPDownloader(progress_interval=1.0, ca_pem=ca, segment_threshold=16 << 20)
    t0 = time.perf_counter()
    c0 = time.process_time()
    await dl.download(d, lambda u, p: None, url)
    wall = time.perf_counter() - t0
    cpu = time.process_time() - c0
    size = os.path.getsize(os.path.join(d, "ab.mkv"))
    os.unlink(os.path.join(d, "ab.mkv"))
    os.rmdir(d)
    await dl.close()
    parent.send("done")
    conns, origin_cpu = parent.recv() if parent.poll(30) else (None, None)
    p.join(30)
    data_len = mib << 20
    ok = size == data_len
    return {"arm": arm, "proto": proto, "bytes": data_len, "wall_s": round(wall, 4),
            "MBps": round(data_len / wall / 1e6, 1), "cpu_s": round(cpu, 4), "ok": ok, "connections": conns,
            "origin_cpu_s": round(origin_cpu, 4) if origin_cpu is not None else None}


async def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--capped-mib", type=int, default=64)
    ap.add_argument("--rate", type=float, default=25e6)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    for arm in ("open", "stream", "conn"):
        for _ in range(a.runs):
            for proto in ("h1", "h2n", "h2n1", "h2"):
                r = await one(arm, proto, a.mib if arm == "open" else a.capped_mib, a.rate)
                rows.append(r)
                print(json.dumps(r), flush=True)
    if a.out:
        os.makedirs(a.out, exist_ok=True)
        with open(os.path.join(a.out, "runs.jsonl"), "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    print("\n| arm | HTTP/1.1 MB/s | HTTP/2 native, 4 conns | native, 1 conn | asyncio, 1 conn | "
          "4 conns / HTTP/1.1 | client CPU s: h1 / 4 conns / 1 conn / asyncio |")
    print("|---|---|---|---|---|---|---|")
    for arm in ("open", "stream", "conn"):
        med = {p: (statistics.median(r["MBps"] for r in rows if r["arm"] == arm and r["proto"] == p),
                   statistics.median(r["cpu_s"] for r in rows if r["arm"] == arm and r["proto"] == p))
               for p in ("h1", "h2n", "h2n1", "h2")}
        print(f"| {arm} | {med['h1'][0]:.1f} | {med['h2n'][0]:.1f} | {med['h2n1'][0]:.1f} | {med['h2'][0]:.1f} | "
              f"{med['h2n'][0] / med['h1'][0]:.2f} | {med['h1'][1]:.3f} / {med['h2n'][1]:.3f} / "
              f"{med['h2n1'][1]:.3f} / {med['h2'][1]:.3f} |")


if __name__ == "__main__":
    asyncio.run(main())
