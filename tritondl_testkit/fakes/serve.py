"""Run one fake backend in its own process (so benches measure the worker,
not the fakes competing for its event loop).

    python -m tritondl_testkit.fakes.serve broker|origin|h2origin|s3 [--port P] [--s3-store discard]
                                   [--tls-cert PEM --tls-key PEM]   # origin / s3 over https
                                   [--variants N --variant-size BYTES]  # per-job payloads
    python -m tritondl_testkit.fakes.serve seed --path FILE_OR_DIR [--piece-kb 1024]

Prints ONE JSON line ``{"kind":..., "endpoint": ..., "url": ...}`` on stdout
once listening, then serves until stdin closes or SIGTERM.  The origin also
serves ``/synthetic/<bytes>/<name>``: deterministic pseudo-random content of
the requested size (generated once per size, cached in memory); a name with
a variant (``movie-3-v7.mkv``) gets that variant's distinct payload, and an
S3 started with ``--variants`` refuses PUTs of variants whose content is not
the origin's (:mod:`tritondl_testkit.fakes.payload`).  ``h2origin`` serves
the same synthetic payloads over HTTP/2 (TLS with ALPN ``h2``; needs
``--tls-cert`` / ``--tls-key``).
"""

from __future__ import annotations

import argparse
import asyncio
import json
import mmap
import os
import signal
import sys

from .broker import Broker
from .h2origin import H2Origin
from .origin import Blob, Origin
from .payload import Expectations, synthetic_bytes, variant_bytes, variant_of
from .s3 import FakeS3

__all__ = ["SyntheticOrigin", "synthetic_bytes"]


class SyntheticOrigin(Origin):
    def __init__(self, *a, **kw) -> None:
        super().__init__(*a, **kw)
        self._cache: dict[tuple[int, int | None], Blob] = {}

    def blob(self, size: int, variant: int | None) -> Blob:
        """The payload as a memfd-backed blob: sendfile serves it, and the bytes
        are held once (in the memfd), not also as a Python object."""
        b = self._cache.get((size, variant))
        if b is None:
            tag = f'"syn-{size}"' if variant is None else f'"syn-{size}-v{variant}"'
            fd = Blob(variant_bytes(size, variant)).fd()
            # the memfd is the one copy: sendfile serves it, and paths that send from
            # user space (https, rate caps) slice a read-only mapping of it
            b = Blob(data=mmap.mmap(fd, size, prot=mmap.PROT_READ) if size else b"", etag=tag)
            b._fd = fd
            self._cache[(size, variant)] = b
        return b

    def precompute(self, size: int, variants: int) -> None:
        """Build every variant's memfd before serving: writing a 10 MiB memfd
        on a job's first request cost that job ~2 ms (r04 fresh-lease run)."""
        for k in range(variants):
            self.blob(size, k)

    async def _handle(self, request):  # type: ignore[override]
        parts = request.path.split("/")
        if len(parts) >= 4 and parts[1] == "synthetic" and parts[2].isdigit():
            self.blobs[request.path] = self.blob(int(parts[2]), variant_of(parts[-1]))
        return await super()._handle(request)


class SyntheticH2Origin(H2Origin):
    """The synthetic payloads of :class:`SyntheticOrigin`, served over HTTP/2."""

    def __init__(self, *a, **kw) -> None:
        super().__init__(*a, **kw)
        self._cache: dict[tuple[int, int | None], tuple[bytes, str, str]] = {}

    def lookup(self, path: str):
        parts = path.split("/")
        if len(parts) >= 4 and parts[1] == "synthetic" and parts[2].isdigit():
            size, variant = int(parts[2]), variant_of(parts[-1])
            b = self._cache.get((size, variant))
            if b is None:
                tag = f'"syn-{size}"' if variant is None else f'"syn-{size}-v{variant}"'
                b = self._cache[(size, variant)] = (variant_bytes(size, variant), tag, "")
            return b
        return super().lookup(path)

    def precompute(self, size: int, variants: int) -> None:
        for k in range(variants):
            self.lookup(f"/synthetic/{size}/x-{k}-v{k}.mkv")


async def _amain(kind: str, port: int, s3_store: str, ak: str | None, sk: str | None,
                 seed_path: str | None = None, piece_kb: int = 1024, encryption: str = "allow",
                 tls_cert: str | None = None, tls_key: str | None = None, rate_mbps: float = 0.0,
                 variants: int = 0, variant_size: int = 0, heartbeat: int = 0) -> None:
    tls = None
    if tls_cert and tls_key:
        with open(tls_cert) as f1, open(tls_key) as f2:
            tls = (f1.read(), f2.read())
    if kind == "seed":
        from tritondl.fetch.bt.torrent import Torrent, TorrentConfig
        from .swarm import magnet_for, torrent_for
        assert seed_path, "--path required"
        info = torrent_for(seed_path, piece_kb << 10)
        cfg = TorrentConfig(listen_host="127.0.0.1", listen_port=port, seed=True, verify_device="cpu", utp=True,
                            encryption=encryption,
                            native_wire=os.environ.get("TRITONDL_BT_NATIVE_WIRE", "1") not in ("0", "false", "off"))
        srv = Torrent(info.infohash, os.path.dirname(os.path.abspath(seed_path)), cfg, info=info)
        await srv.start()
        await srv.download_all()
        info_d = {"kind": kind, "endpoint": f"127.0.0.1:{srv.port}", "url": magnet_for(info),
                  "infohash": info.infohash.hex(), "bytes": info.total_length}
        print(json.dumps(info_d), flush=True)
        loop = asyncio.get_running_loop()
        stop = asyncio.Event()
        for sg in (signal.SIGTERM, signal.SIGINT):
            loop.add_signal_handler(sg, stop.set)
        loop.add_reader(sys.stdin.fileno(), lambda: stop.set() if not os.read(sys.stdin.fileno(), 4096) else None)
        await stop.wait()
        await srv.close()
        return
    if kind == "broker":
        srv = await Broker(port=port, heartbeat=heartbeat).start()
        info = {"kind": kind, "endpoint": srv.endpoint, "url": srv.url}
    elif kind == "origin":
        srv = SyntheticOrigin(port=port, tls=tls)
        if variants and variant_size:
            srv.precompute(variant_size, variants)        # before serving: no job pays for it
        await srv.start()
        info = {"kind": kind, "endpoint": f"{srv.host}:{srv.port}",
                "url": f"{'https' if tls else 'http'}://{srv.host}:{srv.port}"}
    elif kind == "h2origin":
        if tls is None:
            raise SystemExit("h2origin needs --tls-cert and --tls-key")
        srv = SyntheticH2Origin("127.0.0.1", port=port, cert_pem=tls[0], key_pem=tls[1])
        if variants and variant_size:
            srv.precompute(variant_size, variants)
        await srv.start()
        info = {"kind": kind, "endpoint": f"{srv.host}:{srv.port}", "url": f"https://{srv.host}:{srv.port}"}
    elif kind == "s3":
        expect = None
        if variants and variant_size:
            expect = Expectations(variant_size, variants)
            expect.precompute()
        srv = await FakeS3(port=port, store=s3_store, access_key=ak, secret_key=sk, tls=tls, expect=expect).start()
        if rate_mbps:
            srv.rate = rate_mbps * 1e6 / 8
        info = {"kind": kind, "endpoint": srv.endpoint, "url": srv.endpoint}
    else:
        raise SystemExit(f"unknown kind {kind}")
    print(json.dumps(info), flush=True)
    loop = asyncio.get_running_loop()
    stop = asyncio.Event()
    for s in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(s, stop.set)
    loop.add_reader(sys.stdin.fileno(), lambda: stop.set() if not os.read(sys.stdin.fileno(), 4096) else None)
    await stop.wait()
    await srv.stop()


def main() -> None:
    from tritondl.parallel.topology import pin_from_env
    pin_from_env()
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["broker", "origin", "h2origin", "s3", "seed"])
    ap.add_argument("--path", default=None, help="seed: file or directory to seed")
    ap.add_argument("--piece-kb", type=int, default=1024)
    ap.add_argument("--encryption", default="allow", help="seed: MSE policy")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--s3-store", default="discard", choices=["memory", "discard", "disk"])
    ap.add_argument("--access-key", default=None)
    ap.add_argument("--secret-key", default=None)
    ap.add_argument("--tls-cert", default=None, help="origin/s3: serve https with this PEM certificate")
    ap.add_argument("--tls-key", default=None)
    ap.add_argument("--rate-mbps", type=float, default=0.0, help="s3: cap ingest at this many Mbit/s (shared link)")
    ap.add_argument("--variants", type=int, default=0,
                    help="origin: precompute this many payload variants; s3: refuse PUTs of variants whose "
                         "content is not the origin's")
    ap.add_argument("--variant-size", type=int, default=0, help="payload size the variants are precomputed for")
    ap.add_argument("--heartbeat", type=int, default=0, help="broker: heartbeat (s) proposed in connection.tune")
    a = ap.parse_args()
    prof_path = os.environ.get("TRITONDL_FAKE_PROFILE")          # "<path>.<kind>" gets a cProfile dump
    if prof_path:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
        try:
            asyncio.run(_amain(a.kind, a.port, a.s3_store, a.access_key, a.secret_key, a.path, a.piece_kb,
                               a.encryption, a.tls_cert, a.tls_key, a.rate_mbps, a.variants, a.variant_size, a.heartbeat))
        finally:
            prof.disable()
            prof.dump_stats(f"{prof_path}.{a.kind}")
        return
    asyncio.run(_amain(a.kind, a.port, a.s3_store, a.access_key, a.secret_key, a.path, a.piece_kb, a.encryption,
                       a.tls_cert, a.tls_key, a.rate_mbps, a.variants, a.variant_size, a.heartbeat))


if __name__ == "__main__":
    main()
