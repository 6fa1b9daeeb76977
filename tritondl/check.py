"""``python -m tritondl.check`` — preflight of a worker's environment, without
taking a job.

The reference learns that its broker, S3 or work dir are unusable from its
first job (or a ``log.Fatal``, ``cmd/downloader/downloader.go:64-97``).  An
operator moving to this worker can instead check a node or a pod spec
before it joins the queue:

* configuration parses (same variables as the worker; secrets masked);
* native extensions load, and which hashing paths the CPU offers;
* the work dir is writable, its filesystem and free space;
* CPU placement: L3 domains, NUMA nodes, cgroup CPU quota;
* the broker: login, a channel, and a *passive* look at the consume
  exchange, its shard queues and the publish exchange — declares nothing,
  consumes nothing (a 404 / 403 there is reported, with what the worker
  would do about it);
* with ``--lease-probe``, whether this user may hold job leases: a queue
  named and shaped like a lease queue (``<shard>.lease.check-<hex>.0``: TTL,
  dead-letter exchange = the consume exchange, ``x-expires``) is declared
  and deleted at once.  Without that permission the worker holds
  deliveries unacked for the whole job, as the reference did, and a job
  longer than the broker's ``consumer_timeout`` runs again;
* S3: the endpoint parses, which credential provider answers, and a HEAD on
  the bucket (missing is fine: the worker creates it);
* the GPU: visible devices, and with ``--gpu`` the helper process is started
  and pinged (HIP comes up in the helper, never here).

Exit status 0 when nothing failed (warnings allowed), 1 otherwise.
``--json`` prints one JSON document instead of the table.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import tempfile
import time

from .utils.config import Config, parse_args

OK, WARN, FAIL = "ok", "warn", "fail"


class Report:
    def __init__(self) -> None:
        self.items: list[dict] = []

    def add(self, area: str, status: str, detail: str, **extra) -> None:
        self.items.append({"area": area, "status": status, "detail": detail, **extra})

    @property
    def failed(self) -> bool:
        return any(i["status"] == FAIL for i in self.items)


def _mask(v: str) -> str:
    return "" if not v else (v[:2] + "…" if len(v) > 4 else "…")


def check_config(argv: list[str], r: Report) -> Config | None:
    try:
        cfg = Config.from_env(argv=argv)
    except (ValueError, SystemExit) as e:
        r.add("config", FAIL, f"does not parse: {e}")
        return None
    r.add("config", OK, f"consume {cfg.consume_topic} (prefetch {cfg.prefetch}, {cfg.num_shard_queues} shards), "
          f"publish {cfg.publish_topic}, bucket {cfg.bucket}",
          rabbitmq=f"{_mask(cfg.rabbitmq_username)}@{cfg.rabbitmq_endpoint}", s3=cfg.s3_endpoint,
          download_dir=cfg.download_dir)
    if cfg.rabbitmq_endpoint_defaulted:
        r.add("config", WARN, f"RABBITMQ_ENDPOINT not set: the worker will use {cfg.rabbitmq_endpoint}")
    return cfg


def check_native(r: Report) -> None:
    import importlib
    for mod in ("_hash_host", "_relay", "_btwire", "_utp"):
        try:
            importlib.import_module(f"tritondl.{mod}")
            r.add("native", OK, f"{mod} loaded")
        except ImportError as e:
            r.add("native", FAIL, f"{mod} missing ({e}); run python tools/build_native.py")
    try:
        from .ops import hashing
        r.add("native", OK, "16-lane AVX-512 multi-buffer SHA" if hashing.sha_mb()
              else "no AVX-512 multi-buffer SHA on this CPU: SHA-NI / OpenSSL paths")
    except ImportError:
        pass


def mount_of(path: str) -> dict:
    """The mount holding ``path``: {"mnt", "fs", "source"} from the longest
    matching ``/proc/mounts`` entry (fs "?" when unknown)."""
    out = {"mnt": "", "fs": "?", "source": ""}
    try:
        real = os.path.realpath(path)
        with open("/proc/mounts") as m:
            for line in m:
                parts = line.split()
                if len(parts) < 3:
                    continue
                mnt = parts[1]
                inside = real == mnt or real.startswith(mnt.rstrip("/") + "/")
                if inside and len(mnt) >= len(out["mnt"]):
                    out = {"mnt": mnt, "fs": parts[2], "source": parts[0]}
    except OSError:
        pass
    return out


def check_dir(cfg: Config, r: Report) -> None:
    d = cfg.download_dir
    try:
        os.makedirs(d, exist_ok=True)
        with tempfile.NamedTemporaryFile(dir=d, prefix=".tritondl-check-") as f:
            f.write(b"x")
            f.flush()
        st = os.statvfs(d)
        free = st.f_bavail * st.f_frsize
        fs = mount_of(d)["fs"]
        status = OK if free > (1 << 30) else WARN
        r.add("download_dir", status, f"{d} writable, {free / 2**30:.1f} GiB free, filesystem {fs}",
              free_bytes=free, fs=fs)
    except OSError as e:
        r.add("download_dir", FAIL, f"{d}: {e}")


def check_cpus(r: Report) -> None:
    from .parallel import topology
    doms = topology.l3_domains()
    nodes = sorted({topology.numa_node_of(d[0]) for d in doms})
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        quota = None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    detail = f"{sum(len(d) for d in doms)} CPUs in {len(doms)} L3 domain(s) on NUMA node(s) {nodes}"
    if quota is not None:
        detail += f"; cgroup quota {quota:g} CPUs"
    extra: dict = {}
    if len(doms) > 1:
        # other tenants' load per domain, as placement sees it (TRITONDL_CPUS=auto and the pool
        # take idle domains first; a domain another tenant uses slows the jobs pinned there)
        busy = topology.domain_busy(doms)
        idle = sum(1 for b in busy if b <= 0.01)
        detail += f"; {idle} of {len(doms)} L3 domains idle now (placement takes idle ones first)"
        extra["domain_busy"] = {str(d[0]): round(b, 3) for d, b in zip(doms, busy)}
    r.add("cpus", OK, detail, l3_domains=len(doms), numa_nodes=nodes, cpu_quota=quota, **extra)


async def check_broker(cfg: Config, r: Report, timeout: float) -> None:
    from .amqp import codec
    from .amqp.connection import ChannelClosed, Connection
    try:
        conn = await asyncio.wait_for(Connection.open(cfg.rabbitmq_url(), heartbeat=cfg.heartbeat_s), timeout)
    except Exception as e:  # noqa: BLE001 - reported
        r.add("broker", FAIL, f"cannot log in to {cfg.rabbitmq_endpoint}: {e}")
        return
    r.add("broker", OK, f"logged in to {cfg.rabbitmq_endpoint}")
    names = [("exchange", cfg.consume_topic, "declared by the worker at start-up")]
    names += [("queue", f"{cfg.consume_topic}-{i}", "declared by the worker at start-up")
              for i in range(cfg.num_shard_queues)]
    names.append(("exchange", cfg.publish_topic, "the worker declares it best-effort before its first publish"
                  if cfg.declare_publish else "the worker publishes without declaring it (as the reference)"))
    try:
        for kind, name, fix in names:
            ch = await conn.channel()
            try:
                if kind == "exchange":
                    await ch.exchange_declare(name, "direct", passive=True)
                else:
                    await ch.queue_declare(name, passive=True)
                r.add("broker", OK, f"{kind} {name} exists")
            except ChannelClosed as e:
                missing = e.code == codec.NOT_FOUND
                r.add("broker", WARN, f"{kind} {name} {'does not exist' if missing else 'refused'} ({e}); {fix}")
            finally:
                if not ch.is_closed:
                    await ch.close()
    finally:
        await conn.close()


async def check_leases(cfg: Config, r: Report, timeout: float) -> None:
    """Declare and delete one lease-shaped queue (amqp/client.py::_lease_put)."""
    import secrets
    from .amqp.connection import ChannelClosed, Connection
    if cfg.lease_after_s <= 0:
        r.add("leases", OK, "leases are off (TRITONDL_LEASE_AFTER=0): deliveries stay unacked for the whole job")
        return
    name = f"{cfg.consume_topic}-0.lease.check-{secrets.token_hex(4)}.0"
    ms = max(1, int(cfg.lease_s * 1000))
    try:
        conn = await asyncio.wait_for(Connection.open(cfg.rabbitmq_url(), heartbeat=cfg.heartbeat_s), timeout)
    except Exception as e:  # noqa: BLE001 - reported
        r.add("leases", FAIL, f"cannot log in to {cfg.rabbitmq_endpoint}: {e}")
        return
    try:
        ch = await conn.channel()
        try:
            await asyncio.wait_for(ch.queue_declare(name, durable=True, arguments={
                "x-message-ttl": ms, "x-expires": 10_000, "x-dead-letter-exchange": cfg.consume_topic,
                "x-dead-letter-routing-key": f"{cfg.consume_topic}-0"}), timeout)
            await asyncio.wait_for(ch.queue_delete(name), timeout)
            r.add("leases", OK, f"this user may hold job leases (declared and deleted {name}): a job running "
                  f"longer than {cfg.lease_after_s:g} s is leased, whatever the broker's consumer_timeout")
        except ChannelClosed as e:
            r.add("leases", WARN, f"the broker refused a lease queue ({e}): the worker will hold deliveries "
                  "unacked for the whole job, so a job longer than the broker's consumer_timeout runs again. "
                  f"Grant configure and read on '^{cfg.consume_topic}-\\d+\\.lease\\.' and write on the "
                  "default exchange")
        finally:
            if not ch.is_closed:
                await ch.close()
    finally:
        await conn.close()


async def check_s3(cfg: Config, r: Report, timeout: float) -> None:
    from .s3.client import Endpoint, S3Client, S3Error
    from .s3.credentials import default_chain
    try:
        ep = Endpoint.parse(cfg.s3_endpoint)
    except ValueError as e:
        r.add("s3", FAIL, f"S3_ENDPOINT {cfg.s3_endpoint!r} is unusable: {e} (the worker exits at start-up)")
        return
    chain = default_chain()
    v = chain.retrieve()
    who = type(chain._cur).__name__ if chain._cur is not None else "none"
    r.add("s3", OK, f"{'https' if ep.secure else 'http'}://{ep.host}, credentials from {who}"
          + ("" if v.access_key_id else " (anonymous requests)"))
    client = S3Client(cfg.s3_endpoint, chain, region=cfg.s3_region, ca_file=cfg.ca_file)
    try:
        exists = await asyncio.wait_for(client.bucket_exists(cfg.bucket), timeout)
        r.add("s3", OK if exists else WARN, f"bucket {cfg.bucket} " +
              ("exists" if exists else "does not exist yet: the worker creates it (MakeBucket, region \"\")"))
        if client.clock_skew:
            r.add("s3", WARN, f"this host's clock is {client.clock_skew:+.0f} s off S3's: the worker signs on "
                  "S3's clock after its first refused request, but fix the host's time sync", skew_s=client.clock_skew)
    except (S3Error, OSError, asyncio.TimeoutError) as e:
        r.add("s3", FAIL, f"HEAD bucket {cfg.bucket} failed: {e}")
    finally:
        await client.close()


def check_gpu(cfg: Config, r: Report, start_helper: bool) -> None:
    from .ops import hashing
    n = hashing._kfd_gpus()
    if cfg.gpu_verify == "off" or not n:
        r.add("gpu", OK, "no GPU verification (" + ("off" if cfg.gpu_verify == "off" else "no GPU visible")
              + "): resume re-verification hashes on the host")
        return
    r.add("gpu", OK, f"{n} GPU(s) visible; HIP starts only in the verification helper, on first use")
    if start_helper:
        from .ops.gpu_helper import GpuHelper, HelperError
        h = GpuHelper(start_timeout=120)
        t0 = time.monotonic()
        try:
            ok = h.ping()
            r.add("gpu", OK if ok else FAIL, f"helper started and answered in {time.monotonic() - t0:.1f}s")
        except HelperError as e:
            r.add("gpu", FAIL, f"helper: {e}")
        finally:
            h.close()


async def run(argv: list[str], *, timeout: float = 10.0, gpu: bool = False, skip_broker: bool = False,
              skip_s3: bool = False, lease_probe: bool = False) -> Report:
    r = Report()
    cfg = check_config(argv, r)
    check_native(r)
    check_cpus(r)
    if cfg is None:
        return r
    check_dir(cfg, r)
    if not skip_broker:
        await check_broker(cfg, r, timeout)
        if lease_probe:
            await check_leases(cfg, r, timeout)
    if not skip_s3:
        await check_s3(cfg, r, timeout)
    check_gpu(cfg, r, gpu)
    return r


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="python -m tritondl.check", description=__doc__.split("\n\n")[0])
    ap.add_argument("--json", action="store_true", help="one JSON document instead of the table")
    ap.add_argument("--gpu", action="store_true", help="also start the GPU verification helper and ping it")
    ap.add_argument("--timeout", type=float, default=10.0, help="seconds per network check")
    ap.add_argument("--no-broker", action="store_true")
    ap.add_argument("--no-s3", action="store_true")
    ap.add_argument("--lease-probe", action="store_true",
                    help="declare and delete one lease-shaped queue to see whether job leases will work")
    a, rest = ap.parse_known_args(argv)
    parse_args(rest)                                  # the worker's own flags must parse too
    r = asyncio.run(run(rest, timeout=a.timeout, gpu=a.gpu, skip_broker=a.no_broker, skip_s3=a.no_s3,
                        lease_probe=a.lease_probe))
    if a.json:
        print(json.dumps({"ok": not r.failed, "checks": r.items}, indent=1))
    else:
        for i in r.items:
            print(f"{i['status'].upper():4s}  {i['area']:12s}  {i['detail']}")
        print("FAILED" if r.failed else "OK")
    return 1 if r.failed else 0


if __name__ == "__main__":
    sys.exit(main())
