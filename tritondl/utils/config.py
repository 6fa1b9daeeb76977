"""Typed configuration: every env var of the reference under the same name,
plus the reference's hard-coded values as overridable settings whose
defaults equal the reference.

Reference sources: ``cmd/downloader/downloader.go:26,45-58,62,68,81-95,147``,
``internal/rabbitmq/client.go:107-108,308``,
``internal/uploader/uploader.go:25-40``,
``internal/uploader/minio_credential_provider.go:24-30``.
"""

from __future__ import annotations

import argparse
import os
from dataclasses import dataclass, field, fields
from typing import Mapping


def _env_bool(v: str | None, default: bool) -> bool:
    if v is None or v == "":
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


def _default_sign_threads() -> int:
    """aws-chunked chunk hashers per PUT: half the usable CPUs, 2..4.  With
    the 16-lane AVX-512 kernel each hasher claims 16 chunks (1 MiB), so 4
    keep ahead of a download; 8 measured 0.6 ms of CPU per 10 MiB job more
    in waits and wake-ups at no throughput gain (profiles/r03_st_ab/)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 4
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return max(2, min(4, n // 2))


# Worker settings under TRITONDL_<KEY> (values the reference hard-codes, and
# this worker's own knobs): key -> Config field.  docs/CONFIG.md is generated
# from these (tools/gen_config_doc.py) and kept in sync by a test.
ENV_INTS = {"PREFETCH": "prefetch", "CONCURRENCY": "concurrency", "CONCURRENCY_MAX": "concurrency_max", "SHARD_QUEUES": "num_shard_queues",
            "MAX_RETRIES": "max_retries", "BT_LISTEN_PORT": "bt_listen_port", "REDELIVERY_LIMIT": "redelivery_limit",
            "S3_PART_SIZE": "s3_part_size", "S3_MULTIPART_THRESHOLD": "s3_multipart_threshold",
            "S3_PARALLEL_PARTS": "s3_parallel_parts", "HEARTBEAT": "heartbeat_s",
            "HTTP_SEGMENTS": "http_segments", "HTTP_SEGMENT_THRESHOLD": "http_segment_threshold",
            "HTTP2_CONNS": "http2_conns",
            "HTTP_PROBE_BYTES": "http_probe_bytes", "S3_SIGN_THREADS": "s3_sign_threads",
            "HTTP_STRIPE_BYTES": "http_stripe_bytes", "DISK_RESERVE_BYTES": "disk_reserve_bytes",
            "BT_ESTABLISHED_CONNS": "bt_established_conns", "BT_HALF_OPEN_CONNS": "bt_half_open_conns",
            "RECYCLE_BYTES": "recycle_bytes", "MALLOC_MMAP_THRESHOLD": "malloc_mmap_threshold",
            "MALLOC_ARENA_MAX": "malloc_arena_max", "MALLOC_TRIM_THRESHOLD": "malloc_trim_threshold",
            "S3_MAX_RETRIES": "s3_max_retries"}
ENV_FLOATS = {"RETRY_DELAY": "retry_delay_s", "METADATA_TIMEOUT": "metadata_timeout_s",
              "RETRY_BACKOFF": "retry_backoff", "RETRY_DELAY_MAX": "retry_delay_max_s",
              "PROGRESS_INTERVAL": "progress_interval_s", "PROGRESS_LOG_INTERVAL": "progress_log_interval_s",
              "GPU_WARMUP_TIMEOUT": "gpu_warmup_timeout_s", "JOB_LOCK_WAIT": "job_lock_wait_s",
              "MALLOC_TRIM": "malloc_trim_s", "HEALTH_DOWN": "health_down_s", "HEALTH_STALL": "health_stall_s",
              "PIPELINE_COMMIT_MIN_MS": "pipeline_commit_min_ms", "STALE_JOB_DAYS": "stale_job_days",
              "HANDBACK": "handback_s", "LEASE_AFTER": "lease_after_s", "LEASE": "lease_s",
              "S3_RETRY_UNIT": "s3_retry_unit_s", "S3_RETRY_CAP": "s3_retry_cap_s", "S3_STREAM_STALL": "s3_stream_stall_s"}
ENV_STRS = {"CONSUME_TOPIC": "consume_topic", "PUBLISH_TOPIC": "publish_topic", "BUCKET": "bucket",
            "DOWNLOAD_DIR": "download_dir", "DEAD_LETTER_TOPIC": "dead_letter_topic",
            "METRICS_ADDR": "metrics_addr", "GPU_VERIFY": "gpu_verify", "BT_BOOTSTRAP": "bt_bootstrap",
            "BT_ENCRYPTION": "bt_encryption", "CA_FILE": "ca_file", "S3_HASH_DEVICE": "s3_hash_device",
            "CPUS": "cpus"}
ENV_BOOLS = {"CLEANUP": "cleanup", "DROP_FAILED": "drop_failed", "DECLARE_PUBLISH": "declare_publish",
             "DECLARE_PUBLISH_QUEUES": "declare_publish_queues", "STREAM_UPLOAD": "stream_upload",
             "PIPELINE_COMMIT": "pipeline_commit", "BT_DHT": "bt_dht", "BT_DHT_IPV6": "bt_dht_ipv6",
             "BT_UPNP": "bt_upnp", "BT_NATIVE_WIRE": "bt_native_wire", "BT_UTP": "bt_utp", "BT_PEX": "bt_pex",
             "GC_FREEZE": "gc_freeze", "HTTP2": "http2", "H2_NATIVE": "h2_native"}
# The reference's own variables, same names: name -> Config field
REFERENCE_ENV = {"LOG_LEVEL": "log_level", "LOG_FORMAT": "log_format", "RABBITMQ_ENDPOINT": "rabbitmq_endpoint",
                 "RABBITMQ_USERNAME": "rabbitmq_username", "RABBITMQ_PASSWORD": "rabbitmq_password",
                 "S3_ENDPOINT": "s3_endpoint", "S3_ACCESS_KEY": "s3_access_key", "S3_SECRET_KEY": "s3_secret_key",
                 "AWS_ACCESS_KEY_ID": "aws_access_key_id", "AWS_SECRET_ACCESS_KEY": "aws_secret_access_key",
                 "AWS_SESSION_TOKEN": "aws_session_token", "MINIO_ACCESS_KEY": "minio_access_key",
                 "MINIO_SECRET_KEY": "minio_secret_key"}
# Accepted beyond the reference: RABBITMQ_VHOST, S3_REGION, AWS_ACCESS_KEY / AWS_SECRET_KEY (minio-go aliases)
EXTRA_ENV = {"RABBITMQ_VHOST": "rabbitmq_vhost", "S3_REGION": "s3_region",
             "AWS_ACCESS_KEY": "aws_access_key_id", "AWS_SECRET_KEY": "aws_secret_access_key"}


@dataclass
class Config:
    # --- logging / profiling (downloader.go:26,45-52) ---
    cpuprofile: str = ""
    log_level: str = ""
    log_format: str = ""

    # --- broker (downloader.go:54-58, client.go:308) ---
    rabbitmq_endpoint: str = "127.0.0.1:5672"
    rabbitmq_endpoint_defaulted: bool = True
    rabbitmq_username: str = ""
    rabbitmq_password: str = ""
    rabbitmq_vhost: str = "/"
    heartbeat_s: int = 10                       # streadway amqp.Dial's defaultHeartbeat (client.go:309)

    # --- topology (hard-coded in the reference) ---
    consume_topic: str = "v1.download"          # downloader.go:68
    publish_topic: str = "v1.convert"           # downloader.go:147
    num_shard_queues: int = 2                   # client.go:108
    prefetch: int = 1                           # downloader.go:62
    # publish-side topology (the reference declared none, client.go:224): declare the
    # publish exchange (and its shard queues) before the first publish, best-effort —
    # a 403/406 means someone else owns it and the worker publishes without declaring
    declare_publish: bool = True
    declare_publish_queues: bool = True

    # --- job processing ---
    # jobs in flight per process: N > 0 runs exactly N (1 = the reference's one job loop,
    # downloader.go:103); 0 = adaptive, from 1 up to concurrency_max while the jobs mostly
    # wait on the network and the CPUs have room (parallel/adaptive.py: at a 20 ms round
    # trip 4 jobs in flight ran 2.6x the jobs/s of one; on loopback one job keeps the CPUs
    # busy and the limit stays at 1)
    concurrency: int = 0
    # the adaptive limit's cap (job loops started; each holds its streams' executor threads)
    concurrency_max: int = 4
    # a job's publish confirm + ack overlap the next job (service._worker): +30 % at a 2 ms and
    # +47 % at a 20 ms broker round trip, because the confirm's RTT leaves the job's critical
    # path (profiles/r05_rtt_ab/) ...
    pipeline_commit: bool = True
    # ... but on loopback, where a confirm takes ~0.05 ms, the overlap cost ~4 % (372 vs 389
    # jobs/s, profiles/r05_regress/): jobs are pipelined only while the publish -> confirm
    # round trip (EWMA) is at least this long (ms; 0 = always)
    pipeline_commit_min_ms: float = 0.3
    max_retries: int = 5                        # B4 fix: X-Retries budget
    # a job whose delivery keeps coming back unacknowledged (the worker died or lost its
    # channel mid-job: an OOM kill, a crash in native code, a consumer timeout) is
    # dead-lettered once it has been redelivered more than this many times (counted in the
    # job dir, or RabbitMQ's x-delivery-count on quorum queues) instead of taking down
    # every worker that picks it up; 0 = off
    redelivery_limit: int = 5
    retry_delay_s: float = 10.0                 # delivery.go:72 (first retry; waited in a broker delay queue)
    retry_backoff: float = 2.0                  # delay multiplier per retry (1.0 = the reference's fixed 10 s)
    retry_delay_max_s: float = 300.0            # cap on one retry delay
    dead_letter_topic: str = ""                 # "" => "<consume_topic>.dead"
    drop_failed: bool = False                   # opt-out: nack (drop) after max_retries instead of dead-lettering
    # give glibc's free arena memory back to the OS this often (0: never); see Service._trim_heap
    malloc_trim_s: float = 60.0
    # glibc's mmap threshold, fixed (bytes; 0 = glibc's dynamic default).  Dynamic, it
    # climbs to the size of the largest freed block (MiB-sized pump and hash buffers),
    # after which every smaller block lands in a per-thread arena that keeps up to twice
    # that free: a soak's arenas held ~100 MB for 15 MB in use (service.tune_malloc)
    malloc_mmap_threshold: int = 256 * 1024
    malloc_arena_max: int = 0                   # glibc M_ARENA_MAX (0: glibc default, 8 per core)
    # glibc M_TRIM_THRESHOLD, set with a pinned mmap threshold (0: glibc's 128 KiB).  At
    # 128 KiB every free() that leaves more than that at an arena's top returns pages
    # the next allocation faults back: a 200 KiB malloc/free loop took 7x as long
    # (18 faults per cycle); 4 MiB costs ~3 MB of RSS in a soak (profiles/r04_malloc/)
    malloc_trim_threshold: int = 4 << 20
    # move every object alive once the worker is wired (modules, native bindings, torch
    # when the GPU path loaded it: ~180k objects) to CPython's permanent generation before
    # consuming.  A full collection otherwise walks all of them on the event loop: 40-100 ms,
    # a stall in the middle of a job and of the heartbeats (Service.start)
    gc_freeze: bool = True
    # once every job slot has been busy this long (a long download), deliveries buffered
    # behind it (one per other shard consumer) go back to the broker for idle workers and
    # the consumers pause until a slot frees (Client.pause); 0 = hold them (the reference)
    handback_s: float = 60.0
    # with cleanup on: job dirs nothing has touched for this many days and no worker holds
    # (partial downloads of jobs whose message was purged or finished elsewhere) are
    # deleted, at start and hourly; 0 = never (the reference's work dir only grew)
    stale_job_days: float = 7.0
    # a delivery whose job another worker (or another slot of this one) is running waits
    # this long for it, then goes back to the broker (same X-Retries, X-Busy + 1) after a
    # delay that doubles per hand-back from max(1 s, retry_delay_s) up to retry_delay_max_s,
    # instead of pinning an idle job slot for the whole run
    job_lock_wait_s: float = 0.5
    # job leases (amqp.client.Delivery.hold): a job still running this long after its
    # delivery arrived has its delivery acked and a copy kept by the broker in a per-job
    # lease queue instead, renewed every lease_s / 2.  RabbitMQ closes the channel of a
    # delivery left unacked past its consumer_timeout (30 min by default) and requeues it,
    # so another worker would download the job again.  A worker that dies stops renewing:
    # its copy expires after lease_s and goes back to the shard queue.  Needs configure on
    # '<shard>.lease.*' (refused: the delivery is held unacked, the reference's way);
    # 0 = off
    lease_after_s: float = 30.0
    # the lease's TTL: how long a dead worker's job waits in its lease queue before it goes
    # back to the shard queue; renewed every half of it while the job runs
    lease_s: float = 300.0
    # /healthz answers 503 once the broker connection, or the consumer of any shard queue,
    # has been down this long (the supervisor / shard re-subscribe loops keep retrying)
    health_down_s: float = 30.0
    # ... and once this worker has had a free job slot while its shard queues held ready
    # messages for this long without taking one (a consumer that gets nothing; 0 = off)
    health_stall_s: float = 120.0
    # B15: a settled job's dir is deleted (its largest file kept as a spare for the next
    # download, up to recycle_bytes).  The reference never deleted anything, so its work
    # dir grew by every job ever run; TRITONDL_CLEANUP=0 is that behaviour
    cleanup: bool = True
    # with cleanup: keep up to this many bytes of finished job files as spares that new
    # downloads are renamed into and overwrite, instead of freeing and re-allocating
    # their page cache per job (utils/spares.py; 0 = delete every file)
    recycle_bytes: int = 1 << 30
    disk_reserve_bytes: int = 0                 # free-space preflight keeps this much free
    stream_upload: bool = True                  # overlap HTTP fetch with S3 upload
    http_segments: int = 4                      # max parallel Range streams per HTTP file
    http_segment_threshold: int = 64 * 1024 * 1024   # open-ended probe only: segment files at least this big
    http_probe_bytes: int = 0                   # >0: GET probe = bytes=0-(N-1), the rest as parallel Range streams
    # offer HTTP/2 to https origins (ALPN), as grab's Go transport did: the probe and the Range
    # segments become streams, DATA lands in the file from a native session pump, and streams stripe
    # over up to http2_conns connections.  Ties or beats four HTTP/1.1 connections under per-request
    # and per-connection caps with less client CPU (profiles/r06_h2_ab/)
    http2: bool = True
    h2_native: bool = True                      # HTTP/2 DATA via the native session pump (off: asyncio's TLS)
    # HTTP/2 connections per origin: streams go to the least busy one, a new one opens while each
    # carries a stream (four TCP windows, like four HTTP/1.1 connections); 1 = one per origin as Go
    http2_conns: int = 4
    http_stripe_bytes: int = 0                  # >0: parallel streams pull in-order stripes of this size
                                                # (0 measured faster on the 10 MiB headline job: profiles/r01_probe)

    # --- download (downloader.go:81-93, torrent.go:67) ---
    download_dir: str = ""                      # default $CWD/downloading
    progress_interval_s: float = 1.0            # http.go:45, torrent.go:83
    progress_log_interval_s: float = 5.0        # downloader.go:115
    metadata_timeout_s: float = 600.0           # torrent.go:67
    # anacrolix NewDefaultClientConfig defaults (torrent.go:40): ListenPort 42069 (busy →
    # an ephemeral port, see TorrentConfig.listen_port_fallback; 0 = always ephemeral),
    # EstablishedConnsPerTorrent 50, HalfOpenConnsPerTorrent 25
    bt_listen_port: int = 42069
    bt_established_conns: int = 50
    bt_half_open_conns: int = 25
    bt_dht: bool = True
    bt_upnp: bool = True                        # UPnP IGD port forwarding of the listen port (anacrolix default)
    bt_native_wire: bool = True                 # per-block peer-wire work in csrc/btwire (False: pure Python)
    bt_dht_ipv6: bool = True                    # BEP 32 dual-stack DHT (anacrolix default); IPv4-only if no IPv6
    bt_utp: bool = True
    bt_pex: bool = True
    # MSE/PE: disable | allow | prefer | require; anacrolix HeaderObfuscationPolicy{Preferred: true,
    # RequirePreferred: false} = "prefer" (obfuscated first, plaintext accepted)
    bt_encryption: str = "prefer"
    # dht.GlobalBootstrapAddrs (anacrolix/dht v2), in its order
    bt_bootstrap: str = ("router.utorrent.com:6881,router.bittorrent.com:6881,dht.transmissionbt.com:6881,"
                         "dht.aelitis.com:6881,router.silotis.us:6881,dht.libtorrent.org:25401")
    gpu_verify: str = "auto"                    # auto|on|off|hybrid (HIP batch piece hashing; hybrid = GPU + SHA-NI threads)
    gpu_warmup_timeout_s: float = 120.0         # start-up wait for the HIP hasher before consuming

    # --- upload (downloader.go:95, uploader.go) ---
    bucket: str = "triton-staging"
    s3_endpoint: str = ""
    s3_access_key: str = ""
    s3_secret_key: str = ""
    s3_region: str = ""                         # "" => discover per bucket (GET ?location), like minio-go
    # 16 MiB parts: an upload that follows a live download ends ~3 ms after its
    # last byte lands instead of ~11 ms (1 GiB job, profiles/r02_big_ab/); the
    # multipart threshold stays minio-go's 64 MiB, and plan_parts still grows
    # parts to keep any object within 10,000
    s3_part_size: int = 16 * 1024 * 1024
    s3_multipart_threshold: int = 64 * 1024 * 1024
    s3_parallel_parts: int = 4
    # native SHA-256 chunk hashers per streaming PUT: the aws-chunked hashing is on the
    # job's critical path (box A/B, 10 MiB job: 4 -> 245-270, 6 -> 295, 8 -> 307 jobs/s;
    # profiles/r03_st_ab/); half the CPUs this process may use, 2..8
    s3_sign_threads: int = field(default_factory=lambda: _default_sign_threads())
    # where the aws-chunked chunk SHA-256s run: "cpu" (SHA-NI; lowest per-job latency) or
    # "gpu" (the HIP piece kernel, a lane per 64 KiB chunk: ~2.6 ms per batch, so it
    # pays only when the node is CPU-bound, e.g. many workers per CPU share)
    s3_hash_device: str = "cpu"
    # request retries (minio-go retry.go: 10 attempts, 1 s unit, 30 s cap): connection errors,
    # 429/500/502/503/504 and minio's retryable codes (RequestTimeout, SlowDown, ExpiredToken, ...)
    s3_max_retries: int = 9
    # backoff before retry n: unit * 2^n, capped, half of it jittered (the budget spans ~75 s)
    s3_retry_unit_s: float = 1.0
    # the longest wait between two attempts
    s3_retry_cap_s: float = 30.0
    # a streamed PUT (the upload following its download) gives up after the download made no
    # progress for this long, and the file is uploaded once the download is done: S3 answers
    # 400 RequestTimeout to a request body that sends nothing for ~20 s (0 = follow forever)
    s3_stream_stall_s: float = 10.0
    aws_access_key_id: str = ""
    aws_secret_access_key: str = ""
    aws_session_token: str = ""
    minio_access_key: str = ""
    minio_secret_key: str = ""

    # --- TLS trust (https origins / S3): "" = system store (SSL_CERT_FILE honoured) ---
    ca_file: str = ""

    # --- placement ---
    # CPU set the worker pins itself to at start-up: a cpulist ("0-7,128-135"),
    # "auto" (one whole L3 domain: a lone worker the idlest one, else the
    # LOCAL_RANK-th of LOCAL_WORLD_SIZE spread evenly over the node), "auto:N" (N CPUs packed into the fewest L3
    # domains) or "" (no pinning; the pool sets a cpulist per worker).  One CCD
    # keeps a job's bytes in its L3 as they pass receive pump -> hashers ->
    # send pump (profiles/r03_pin_ab/)
    cpus: str = ""

    # --- observability ---
    metrics_addr: str = ""                      # "host:port" → /metrics
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_env(cls, env: Mapping[str, str] | None = None, argv: list[str] | None = None) -> "Config":
        env = os.environ if env is None else env
        c = cls()
        g = env.get
        c.log_level = g("LOG_LEVEL", "")
        c.log_format = g("LOG_FORMAT", "")
        ep = g("RABBITMQ_ENDPOINT", "")
        if ep:
            c.rabbitmq_endpoint, c.rabbitmq_endpoint_defaulted = ep, False
        c.rabbitmq_username = g("RABBITMQ_USERNAME", "")
        c.rabbitmq_password = g("RABBITMQ_PASSWORD", "")
        c.rabbitmq_vhost = g("RABBITMQ_VHOST", "/") or "/"
        c.s3_endpoint = g("S3_ENDPOINT", "")
        c.s3_access_key = g("S3_ACCESS_KEY", "")
        c.s3_secret_key = g("S3_SECRET_KEY", "")
        c.s3_region = g("S3_REGION", c.s3_region) or c.s3_region
        c.aws_access_key_id = g("AWS_ACCESS_KEY_ID", "") or g("AWS_ACCESS_KEY", "")
        c.aws_secret_access_key = g("AWS_SECRET_ACCESS_KEY", "") or g("AWS_SECRET_KEY", "")
        c.aws_session_token = g("AWS_SESSION_TOKEN", "")
        c.minio_access_key = g("MINIO_ACCESS_KEY", "")
        c.minio_secret_key = g("MINIO_SECRET_KEY", "")
        # Extensions (TRITONDL_*) for values the reference hard-codes.
        for k, a in ENV_INTS.items():
            if g("TRITONDL_" + k):
                setattr(c, a, int(g("TRITONDL_" + k)))
        for k, a in ENV_FLOATS.items():
            if g("TRITONDL_" + k):
                setattr(c, a, float(g("TRITONDL_" + k)))
        for k, a in ENV_STRS.items():
            if g("TRITONDL_" + k) is not None and g("TRITONDL_" + k) != "":
                setattr(c, a, g("TRITONDL_" + k))
        for k, a in ENV_BOOLS.items():
            setattr(c, a, _env_bool(g("TRITONDL_" + k), getattr(c, a)))
        if c.s3_hash_device not in ("cpu", "gpu"):
            raise ValueError(f"TRITONDL_S3_HASH_DEVICE must be cpu|gpu, got {c.s3_hash_device!r}")
        if c.bt_encryption not in ("disable", "allow", "prefer", "require"):
            raise ValueError(f"TRITONDL_BT_ENCRYPTION must be disable|allow|prefer|require, got {c.bt_encryption!r}")
        if argv is not None:
            c.apply_args(parse_args(argv))
        if not c.download_dir:
            c.download_dir = os.path.join(os.getcwd(), "downloading")
        return c

    def apply_args(self, ns: argparse.Namespace) -> None:
        for f in fields(self):
            v = getattr(ns, f.name, None)
            if v is not None:
                setattr(self, f.name, v)

    @property
    def dlq_topic(self) -> str:
        """Where a job goes after ``max_retries`` (never dropped unless ``drop_failed``)."""
        return self.dead_letter_topic or f"{self.consume_topic}.dead"

    def retry_delay_for(self, retries: int) -> float:
        """Delay before retry number ``retries + 1``: ``retry_delay_s`` growing by
        ``retry_backoff`` per retry, capped at ``retry_delay_max_s``."""
        if self.retry_delay_s <= 0:
            return 0.0
        return min(self.retry_delay_max_s, self.retry_delay_s * self.retry_backoff ** max(0, retries))

    def rabbitmq_url(self) -> str:
        """amqp://user:pass@endpoint/vhost with credentials URL-escaped (B14 fix)."""
        from urllib.parse import quote
        user = quote(self.rabbitmq_username, safe="")
        pw = quote(self.rabbitmq_password, safe="")
        vh = "" if self.rabbitmq_vhost == "/" else "/" + quote(self.rabbitmq_vhost, safe="")
        return f"amqp://{user}:{pw}@{self.rabbitmq_endpoint}{vh}"


def build_arg_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="tritondl", description="media ingest worker (downloader-go capabilities)")
    # Go's flag package accepts both -cpuprofile and --cpuprofile.
    p.add_argument("-cpuprofile", "--cpuprofile", dest="cpuprofile", default=None,
                   help="write cpu profile to file")
    p.add_argument("--concurrency", type=int, default=None,
                   help="jobs in flight per process (0: adaptive, the default; reference: 1)")
    p.add_argument("--prefetch", type=int, default=None, help="AMQP QoS prefetch (reference: 1)")
    p.add_argument("--download-dir", dest="download_dir", default=None)
    p.add_argument("--bucket", default=None)
    p.add_argument("--consume-topic", dest="consume_topic", default=None)
    p.add_argument("--publish-topic", dest="publish_topic", default=None)
    p.add_argument("--metrics-addr", dest="metrics_addr", default=None)
    p.add_argument("--cleanup", dest="cleanup", action="store_true", default=None)
    p.add_argument("--gpu-verify", dest="gpu_verify", choices=["auto", "on", "off", "hybrid"], default=None)
    return p


def parse_args(argv: list[str]) -> argparse.Namespace:
    return build_arg_parser().parse_args(argv)
