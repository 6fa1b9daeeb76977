#!/usr/bin/env python3
"""BitTorrent ingest benchmark ("Magnet job against a local
seeder swarm"): N seeder processes on 127.0.0.1 serve one synthetic file; the
leecher (this process, the production TorrentDownloader) downloads it from a
magnet with x.pe peers.  Prints one JSON line with MB/s.

    python tools/bench_bt.py --mb 1024 --seeds 4 [--utp] [--piece-kb 1024]
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


async def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=512)
    ap.add_argument("--seeds", type=int, default=4)
    ap.add_argument("--piece-kb", type=int, default=1024)
    ap.add_argument("--utp", action="store_true", help="disable TCP dialing: uTP only")
    ap.add_argument("--profile", default="")
    ap.add_argument("--encryption", default="allow", help="MSE policy for seeders and leecher")
    a = ap.parse_args()
    from tritondl.bench_job import Backend
    from tritondl.fakes.swarm import make_payload
    from tritondl.fetch.bt.client import TorrentDownloader
    from tritondl.fetch.bt.metainfo import parse_magnet
    from tritondl.fetch.bt.torrent import Torrent, TorrentConfig
    from tritondl.utils.log import log
    log.configure("warning", "")
    td = tempfile.mkdtemp(prefix="tdl-btbench-", dir=os.environ.get("TMPDIR", "/tmp"))
    seeds = []
    try:
        src = os.path.join(td, "src")
        make_payload(src, {"movie.mkv": a.mb << 20})
        seeds = [await Backend("seed", ["--path", os.path.join(src, "movie.mkv"), "--piece-kb",
                                        str(a.piece_kb), "--encryption", a.encryption]).start()
                 for _ in range(a.seeds)]
        magnet = seeds[0].info["url"]
        peers = "&".join(f"x.pe={s.info['endpoint']}" for s in seeds)
        magnet = magnet + "&" + peers
        if a.utp:
            async def no_tcp(self, addr):
                raise OSError("tcp disabled")
            Torrent._dial_tcp = no_tcp  # type: ignore[assignment]
        dst = os.path.join(td, "dst")
        os.makedirs(dst)
        d = TorrentDownloader(TorrentConfig(listen_host="127.0.0.1", verify_device="cpu", utp=True,
                                            encryption=a.encryption),
                              progress_interval=1.0, use_dht=False)
        prof = None
        if a.profile:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        await d.download(dst, lambda u, p: None, magnet)
        dt = time.perf_counter() - t0
        if prof:
            prof.disable()
            prof.dump_stats(a.profile)
        assert parse_magnet(magnet).infohash.hex() == seeds[0].info["infohash"]
        assert os.path.getsize(os.path.join(dst, "movie.mkv")) == a.mb << 20
        print(json.dumps({"metric": "bt_ingest_MB_per_sec", "value": round(a.mb * 1.048576 / dt, 1),
                          "seconds": round(dt, 3), "mb": a.mb, "seeds": a.seeds, "piece_kb": a.piece_kb,
                          "transport": "utp" if a.utp else "tcp+utp",
                          "encryption": a.encryption}), flush=True)
    finally:
        for s in seeds:
            await s.stop()
        shutil.rmtree(td, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(asyncio.run(main()))
