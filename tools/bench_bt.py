#!/usr/bin/env python3
"""BitTorrent ingest benchmark ("Magnet job against a local
seeder swarm"): N seeder processes on 127.0.0.1 serve one synthetic file; the
leecher (this process, the production TorrentDownloader) downloads it from a
magnet with x.pe peers.  Prints one JSON line with MB/s.

    python tools/bench_bt.py --mb 1024 --seeds 4 [--utp] [--piece-kb 1024]

``--job``: the whole worker job instead of the bare download — a multi-file
season pack (``--files`` media files sharing ``--mb``) published as a magnet
``v1.download`` job on a fake broker, run by the production ``Service``
(torrent download → select → S3 multipart upload to a fake S3 → publish →
ack), timed from publish to ack.  ``--stream both`` runs it with per-file
streamed uploads off (the reference's order: upload after the whole torrent)
and on, alternating, and prints one JSON line per run.
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
    ap.add_argument("--cpuprofile", default="", help="whole-process sampling profile (pprof + .txt) of the download")
    ap.add_argument("--encryption", default="allow", help="MSE policy for seeders and leecher")
    ap.add_argument("--job", action="store_true", help="full worker job (download+upload+publish+ack)")
    ap.add_argument("--python-seeders", action="store_true",
                    help="seeders answer REQUESTs in Python instead of the native link")
    ap.add_argument("--python-wire", action="store_true",
                    help="leecher: per-block work in Python instead of the native csrc/btwire link")
    ap.add_argument("--files", type=int, default=8, help="--job: media files in the pack")
    ap.add_argument("--stream", default="both", choices=["on", "off", "both"])
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--s3-gbps", type=float, default=0.0,
                    help="--job: cap the fake S3's ingest link (Gbit/s; 0 = loopback speed)")
    ap.add_argument("--cpus", default="", help="pin the leecher (worker) to this cpulist")
    ap.add_argument("--fake-cpus", default="", help="pin the seeder (and fake S3) processes to this cpulist")
    ap.add_argument("--malloc-trim-threshold", type=int, default=-1,
                    help="glibc trim threshold with a pinned mmap threshold (0: glibc's 128 KiB; -1: worker default)")
    ap.add_argument("--malloc-mmap-threshold", type=int, default=-1,
                    help="glibc mmap threshold for the leecher (0: glibc's dynamic default; -1: the worker "
                         "default, which the plain download form leaves to glibc)")
    a = ap.parse_args()
    if a.fake_cpus:
        os.environ["TRITONDL_BENCH_FAKE_CPUS"] = a.fake_cpus   # the fakes pin themselves (topology.pin_from_env)
    if a.cpus:
        from tritondl.parallel.topology import parse_cpulist
        os.sched_setaffinity(0, parse_cpulist(a.cpus))
    if a.python_seeders:
        os.environ["TRITONDL_BT_NATIVE_WIRE"] = "0"     # read by the seeder processes (fakes/serve.py)
    if a.job:
        return await job_bench(a)
    if a.malloc_mmap_threshold > 0:
        from tritondl.service import tune_malloc
        from tritondl.utils.config import Config
        tune_malloc(a.malloc_mmap_threshold, trim_threshold=(a.malloc_trim_threshold if a.malloc_trim_threshold >= 0
                                                             else Config().malloc_trim_threshold))
    from tritondl_testkit.bench_job import Backend
    from tritondl_testkit.fakes.swarm import make_payload
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
                                            encryption=a.encryption, native_wire=not a.python_wire),
                              progress_interval=1.0, use_dht=False)
        prof = sprof = None
        if a.profile:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        if a.cpuprofile:
            from tritondl.utils.profiler import CPUProfiler
            sprof = CPUProfiler(a.cpuprofile)
            sprof.start()
        import resource
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        await d.download(dst, lambda u, p: None, magnet)
        dt = time.perf_counter() - t0
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        if prof:
            prof.disable()
            prof.dump_stats(a.profile)
        if sprof:
            sprof.stop()                                 # writes PATH and PATH.txt
        assert parse_magnet(magnet).infohash.hex() == seeds[0].info["infohash"]
        assert os.path.getsize(os.path.join(dst, "movie.mkv")) == a.mb << 20
        print(json.dumps({"metric": "bt_ingest_MB_per_sec", "value": round(a.mb * 1.048576 / dt, 1),
                          "seconds": round(dt, 3), "mb": a.mb, "seeds": a.seeds, "piece_kb": a.piece_kb,
                          "transport": "utp" if a.utp else "tcp+utp",
                          "encryption": a.encryption, "wire": "python" if a.python_wire else "native",
                          "seeders": "python" if a.python_seeders else "native",
                          # the leecher process over the download: page faults and CPU
                          "leecher_minflt": ru1.ru_minflt - ru0.ru_minflt,
                          "leecher_cpu_s": round(ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime, 3)}),
              flush=True)
    finally:
        for s in seeds:
            await s.stop()
        shutil.rmtree(td, ignore_errors=True)
    return 0


async def job_bench(a) -> int:
    from tritondl.amqp.client import Client
    from tritondl.amqp.codec import Properties
    from tritondl.amqp.connection import Connection
    from tritondl_testkit.bench_job import AK, SK, Backend
    from tritondl_testkit.fakes.swarm import make_payload
    from tritondl.fetch.bt.client import TorrentDownloader
    from tritondl.fetch.bt.torrent import TorrentConfig
    from tritondl.fetch.registry import Dispatcher
    from tritondl.models import Download, Media, SourceType
    from tritondl.s3.client import S3Client
    from tritondl.s3.credentials import Static
    from tritondl.s3.uploader import Uploader
    from tritondl.service import Service
    from tritondl.utils.config import Config
    from tritondl.utils.log import log
    log.configure("warning", "")
    td = tempfile.mkdtemp(prefix="tdl-btjob-", dir=os.environ.get("TMPDIR", "/tmp"))
    backs = []
    svc = None
    prod = None
    try:
        pack = os.path.join(td, "src", "Show.S01")
        per = (a.mb << 20) // a.files
        make_payload(pack, {f"season 1/e{k + 1:02d}.mkv": per for k in range(a.files)} | {"info.nfo": 4096})
        seeds = [await Backend("seed", ["--path", pack, "--piece-kb", str(a.piece_kb),
                                        "--encryption", a.encryption]).start() for _ in range(a.seeds)]
        broker = await Backend("broker").start()
        s3 = await Backend("s3", ["--s3-store", "discard", "--access-key", AK, "--secret-key", SK,
                                  "--rate-mbps", str(a.s3_gbps * 1000)]).start()
        backs = seeds + [broker, s3]
        magnet = seeds[0].info["url"] + "&" + "&".join(f"x.pe={s.info['endpoint']}" for s in seeds)
        cfg = Config()
        cfg.download_dir = os.path.join(td, "downloading")
        cfg.cleanup, cfg.max_retries, cfg.retry_delay_s = True, 0, 0.0
        cfg.recycle_bytes = int(os.environ.get("TRITONDL_RECYCLE_BYTES", cfg.recycle_bytes))
        cfg.progress_log_interval_s, cfg.heartbeat_s = 0, 0
        if a.malloc_mmap_threshold >= 0:
            cfg.malloc_mmap_threshold = a.malloc_mmap_threshold
        if a.malloc_trim_threshold >= 0:
            cfg.malloc_trim_threshold = a.malloc_trim_threshold
        bt = TorrentDownloader(TorrentConfig(listen_host="127.0.0.1", verify_device="cpu", utp=True,
                                             encryption=a.encryption, native_wire=not a.python_wire),
                               progress_interval=1.0, use_dht=False)
        svc = Service(cfg, amqp=Client(broker.info["url"], heartbeat=0, retry_delay=0),
                      dispatcher=Dispatcher(cfg.download_dir, [bt], 0),
                      uploader=Uploader(cfg.bucket, S3Client(s3.info["url"], Static(AK, SK))))
        await svc.start()
        prod = await Connection.open(broker.info["url"], heartbeat=0)
        ch = await prod.channel()
        await ch.confirm_select()
        modes = {"on": [True], "off": [False], "both": [False, True]}[a.stream]
        for rep in range(a.repeat):
            for on in modes:
                cfg.stream_upload = on
                n0 = svc.jobs_finished
                body = Download(created_at="now", media=Media(id=f"pack-{rep}-{int(on)}", source=SourceType.TORRENT,
                                                              source_uri=magnet)).encode()
                t0 = time.perf_counter()
                await ch.basic_publish("v1.download", "v1.download-0", body, Properties(delivery_mode=2))
                await svc.wait_finished(n0 + 1, timeout=600)
                dt = time.perf_counter() - t0
                r = svc.results[-1]
                assert r.ok and r.files == a.files and r.bytes == per * a.files, r
                print(json.dumps({"metric": "bt_job_seconds", "value": round(dt, 3), "stream_upload": on,
                                  "s3_link_gbps": a.s3_gbps or None, "wire": "python" if a.python_wire else "native",
                                  "seeders": "python" if a.python_seeders else "native",
                                  "mb": a.mb, "files": a.files, "seeds": a.seeds, "piece_kb": a.piece_kb,
                                  "job_MB_per_sec": round(a.mb * 1.048576 / dt, 1),
                                  "spans_ms": {k: round(v * 1000, 1) for k, v in r.marks.items()}}), flush=True)
    finally:
        if prod is not None:
            await prod.close()
        if svc is not None:
            await svc.shutdown(grace=10)
        for b in backs:
            await b.stop()
        shutil.rmtree(td, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(asyncio.run(main()))
