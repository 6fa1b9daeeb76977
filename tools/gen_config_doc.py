#!/usr/bin/env python3
"""Generate docs/CONFIG.md: every environment variable the worker reads.

Sources of truth:
* the reference's own variables and the ``TRITONDL_*`` worker settings come
  from ``tritondl/utils/config.py`` (``REFERENCE_ENV``, ``EXTRA_ENV``,
  ``ENV_*`` maps; defaults from ``Config()``; descriptions from the comments
  on the dataclass fields);
* process-level knobs read directly by a module (hashing, data plane,
  profiler, ...) are listed in ``DIRECT`` below.

``tests/test_config_doc.py`` fails when the file is stale or when any
``TRITONDL_*`` name in ``tritondl/`` or ``csrc/`` is missing from it.

    python tools/gen_config_doc.py            # rewrite docs/CONFIG.md
    python tools/gen_config_doc.py --check    # exit 1 if it is out of date
"""

from __future__ import annotations

import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "docs", "CONFIG.md")

# name -> (default, where it is read, what it does)
DIRECT = {
    "TRITONDL_MEDIA_FIELDS": ("id=1,…", "models/messages.py",
                              "field numbers of `api.Media` (the schema is a reconstruction)"),
    "TRITONDL_ENVELOPE_FIELDS": ("created_at=1,media=2", "models/messages.py",
                                 "field numbers of `api.Download` / `api.Convert`"),
    "TRITONDL_GPU_HELPER": ("1", "ops/hashing.py",
                            "0: GPU verification in the worker process instead of the idle-exiting helper"),
    "TRITONDL_GPU_IDLE_S": ("30", "ops/hashing.py",
                            "the helper exits (and an in-process hasher frees HBM + pinned stages) after this long idle"),
    "TRITONDL_GPU_MAX_HBM": ("8 GiB", "ops/hashing.py, hip/gpu_hash.hip", "cap on the hasher's two HBM windows"),
    "TRITONDL_GPU_CALL_TIMEOUT": ("120", "ops/gpu_helper.py",
                                  "seconds a helper call may go without progress (bytes read) before the helper is "
                                  "killed; `auto` then hashes that batch on the host"),
    "TRITONDL_GPU_COOLDOWN_S": ("600", "ops/hashing.py",
                                "after 3 consecutive failed GPU calls (or a helper that cannot start) `auto` "
                                "hashes on the host for this long, then offers the GPU again"),
    "TRITONDL_GPU_PROGRESS_S": ("1", "ops/gpu_helper.py", "interval of the helper's progress heartbeat during a call"),
    "TRITONDL_TLS_SEND_MAP": ("1", "relay/relay_core.h",
                              "0: TLS uploads pread into a buffer instead of encrypting from a mapping of the file"),
    "TRITONDL_GPU_DEVICE": ("LOCAL_RANK or 0", "ops/hashing.py", "the worker's GPU"),
    "TRITONDL_GPU_DIRECT": ("1", "ops/hashing.py, hip/gpu_hash.hip",
                            "0: stage piece data through pinned host buffers instead of DMA from the page cache"),
    "TRITONDL_GPU_DIRECT_BLOCK_MB": ("256", "hip/gpu_hash.hip", "registered-mapping block size of the direct DMA path"),
    "TRITONDL_GPU_DIRECT_KEEP": ("unset", "hip/gpu_hash.hip", "keep direct-DMA registrations between batches"),
    "TRITONDL_GPU_READERS": ("4", "ops/hashing.py", "pread threads filling the staging ring (staged path)"),
    "TRITONDL_GPU_STAGE_MB": ("128", "ops/hashing.py", "size of one pinned staging slot (ring of 4)"),
    "TRITONDL_GPU_WARMUP": ("unset", "ops/hashing.py", "1: start the GPU hasher at worker start-up"),
    "TRITONDL_GPU_TRACE": ("unset", "ops/hashing.py", "1: per-batch timing trace of the GPU hasher"),
    "TRITONDL_HYBRID_CPU_THREADS": ("CPUs − 1", "ops/hashing.py", "host hashing threads beside the GPU in hybrid verify"),
    "TRITONDL_SHA_MB": ("1", "hash/sha256_mb.h, hash/hash_host.cpp", "0: no 16-lane AVX-512 multi-buffer SHA"),
    "TRITONDL_SHA_MB_HEAD": ("0", "relay/relay_core.h", "chunks hashed one by one before the multi-buffer groups start"),
    "TRITONDL_SHA_MB_TAIL": ("32", "relay/relay_core.h", "chunks at a PUT's end hashed one by one (tail latency)"),
    "TRITONDL_SHA_MB_FOLLOW": ("1", "relay/relay_core.h",
                               "streamed signed PUT: 16-chunk hash claims only over bytes already downloaded "
                               "(0: by position)"),
    "TRITONDL_S3_CHUNK_KB": ("64", "s3/sigv4.py",
                             "aws-chunked payload chunk of a signed streaming PUT (minio-go's 64 KiB; 8 and up)"),
    "TRITONDL_ZC_TRACE": ("0", "relay/relay_core.h",
                          "1: one timing line per signed PUT on stderr (when each chunk landed, was hashed, was sent)"),
    "TRITONDL_ZC_POPULATE": ("0", "relay/relay_core.h",
                             "1: map a signed PUT's whole file mapping up front (MADV_POPULATE_READ) "
                             "instead of a minor fault per page"),
    "TRITONDL_ZC_WRITE_BATCH": ("0", "relay/relay_core.h",
                                "signed plain-http PUT: ready frames per writev from the file mapping "
                                "(0/1: a header send + sendfile per 64 KiB frame)"),
    "TRITONDL_SHA_NI": ("1", "hash/sha_ni.h, hash/hash_host.cpp", "0: OpenSSL instead of the two-stream SHA-NI path"),
    "TRITONDL_NATIVE_RELAY": ("1", "utils/rawhttp.py", "0: aiohttp data plane instead of the native pumps"),
    "TRITONDL_RELAY_PORT": ("0", "utils/rawhttp.py", "1: pumps post to a completion port instead of executor threads"),
    "TRITONDL_RELAY_SPLICE": ("0", "fetch/http.py", "1: splice(2) receive (slower with parallel ranges on overlayfs)"),
    "TRITONDL_RELAY_RECV_BUF": ("4 MiB", "fetch/http.py", "receive pump buffer"),
    "TRITONDL_RELAY_ZC": ("1", "relay/relay_core.h", "0: ring-buffer chunked PUTs instead of zero-copy"),
    "TRITONDL_TRACE": ("unset", "utils/rawhttp.py", "1: record data-plane events (diagnostics)"),
    "TRITONDL_PROFILE_HZ": ("100", "utils/profiler.py", "sampling rate of `-cpuprofile`"),
}
# notes for settings whose field carries no comment of its own
NOTES = {
    "log_level": "`debug`: caller reporting (the reference's only effect) and debug level (B10); `downloader.go:45-47`",
    "log_format": "`json`: JSON lines; `downloader.go:49-52`",
    "rabbitmq_endpoint": "host:port; unset → warning and the default (`downloader.go:54-58`)",
    "rabbitmq_username": "put URL-escaped into `amqp://user:pass@endpoint` (B14 fix; `client.go:308`)",
    "rabbitmq_password": "as `RABBITMQ_USERNAME`",
    "s3_endpoint": "URL; `https` → TLS (`uploader.go:25-40`); unusable → fatal at start-up",
    "s3_access_key": "with `S3_SECRET_KEY`: SigV4, else the next provider (`minio_credential_provider.go:24-30`)",
    "s3_secret_key": "as `S3_ACCESS_KEY`",
    "aws_access_key_id": "credential chain fallback (`credentials.EnvAWS`, `uploader.go:45-49`)",
    "aws_secret_access_key": "as `AWS_ACCESS_KEY_ID`",
    "aws_session_token": "sent as `x-amz-security-token` with the AWS keys",
    "minio_access_key": "credential chain fallback (`credentials.EnvMinio`)",
    "minio_secret_key": "as `MINIO_ACCESS_KEY`",
    "bt_dht": "BEP 5 DHT peer discovery (anacrolix default)",
    "bt_established_conns": "anacrolix EstablishedConnsPerTorrent",
    "bt_half_open_conns": "anacrolix HalfOpenConnsPerTorrent",
    "bt_pex": "BEP 11 peer exchange (never for private torrents)",
    "bt_utp": "uTP (BEP 29) beside TCP on the same port",
    "bucket": "`downloader.go:95`",
    "ca_file": "extra CA bundle for https origins / S3 (\"\": the system store, `SSL_CERT_FILE` honoured)",
    "declare_publish_queues": "with `DECLARE_PUBLISH`: also declare and bind `<topic>-0..N-1`",
    "s3_multipart_threshold": "objects at least this big go multipart (minio-go's 64 MiB)",
    "s3_parallel_parts": "multipart parts in flight per object",
}
# bench / test harness only (never read by a production worker)
HARNESS = {
    "TRITONDL_BENCH_FAKE_CPUS": "CPU set the bench's fake endpoints pin themselves to (set by `bench.py`)",
    "TRITONDL_BENCH_DOMAIN_BUSY": "busy share of the rank's CCD at launch (set by `bench.py`, reported in `config`)",
    "TRITONDL_BENCH_LOOP_PROFILE": "cProfile of the event-loop thread over the timed jobs (`bench.py`)",
    "TRITONDL_FAKE_S3_VERIFY_THREADS": "aws-chunked verifier threads per PUT in the fake S3 (default 4)",
    "TRITONDL_FAKE_PROFILE": "cProfile dump of a fake endpoint process",
    "TRITONDL_GPU_HELPER_FAKE": "tests: a host stand-in for the GPU helper's hasher",
    "TRITONDL_GPU_HELPER_FAKE_STALL": "tests: seconds the stand-in helper stalls per call",
    "TRITONDL_GPU_HELPER_FAKE_SLOW": "tests: seconds the stand-in helper takes per call while reporting progress",
    "TRITONDL_FAKE_RTT_MS": "emulated round trip of the fake broker / origin / S3 (set by `bench.py --rtt-ms`)",
    "TRITONDL_FAKE_STREAM_MBPS": "per-stream bandwidth cap of the fake origin / S3 (set by `bench.py --stream-mbps`)",
    "TRITONDL_GPU_HELPER_CHILD": "internal: set in the helper process itself",
}


def _field_docs() -> dict[str, str]:
    """Config field -> its comment (trailing, else the comment lines above)."""
    path = os.path.join(ROOT, "tritondl", "utils", "config.py")
    src = open(path).read()
    lines = src.splitlines()
    tree = ast.parse(src)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Config")
    out: dict[str, str] = {}
    for node in cls.body:
        if not isinstance(node, ast.AnnAssign) or not isinstance(node.target, ast.Name):
            continue
        line = lines[node.lineno - 1]
        text = ""
        if "#" in line.split("=", 1)[-1]:
            text = line.split("#", 1)[1].strip()
        above = []
        i = node.lineno - 2
        while i >= 0 and lines[i].strip().startswith("#") and not lines[i].strip().startswith("# ---"):
            above.insert(0, lines[i].strip().lstrip("#").strip())
            i -= 1
        if above:
            text = (" ".join(above) + ("; " + text if text else "")).strip()
        out[node.target.id] = text.replace("|", "\\|")
    return out


def _default(cfg, name: str) -> str:
    v = getattr(cfg, name)
    if name == "s3_sign_threads":
        return "half the CPUs, 2..4"
    if isinstance(v, bool):
        return "on" if v else "off"
    if isinstance(v, str):
        return f"`{v}`" if v else '""'
    return f"`{v}`"


def render() -> str:
    from tritondl.utils import config as C
    cfg = C.Config()
    docs = _field_docs()
    out = ["# Configuration", "",
           "Every environment variable the worker reads.  Generated by `tools/gen_config_doc.py` from",
           "`tritondl/utils/config.py` (and the module-level knobs listed there); `tests/test_config_doc.py`",
           "keeps it complete.  Defaults equal the reference's values wherever the reference had one",
           "(SURVEY.md §5.6).  `python -m tritondl --help` lists the command-line flags.", "",
           "## The reference's variables (same names)", "",
           "| variable | setting | default | notes |", "|---|---|---|---|"]
    for var, f in C.REFERENCE_ENV.items():
        out.append(f"| `{var}` | `{f}` | {_default(cfg, f)} | {docs.get(f) or NOTES.get(f, '')} |")
    out += ["", "Also accepted (not read by the reference):", "",
            "| variable | setting |", "|---|---|"]
    for var, f in C.EXTRA_ENV.items():
        out.append(f"| `{var}` | `{f}` |")
    out += ["", "## Worker settings (`TRITONDL_<KEY>`)", "",
            "Values the reference hard-codes, and this worker's own settings.", "",
            "| variable | type | setting | default | notes |", "|---|---|---|---|---|"]
    rows = []
    for typ, m in (("int", C.ENV_INTS), ("float", C.ENV_FLOATS), ("str", C.ENV_STRS), ("bool", C.ENV_BOOLS)):
        for k, f in m.items():
            rows.append((k, typ, f))
    for k, typ, f in sorted(rows):
        out.append(f"| `TRITONDL_{k}` | {typ} | `{f}` | {_default(cfg, f)} | {docs.get(f) or NOTES.get(f, '')} |")
    out += ["", "## Process-level knobs (read directly by a module)", "",
            "| variable | default | read in | effect |", "|---|---|---|---|"]
    for var, (dflt, where, what) in sorted(DIRECT.items()):
        out.append(f"| `{var}` | {dflt} | `{where}` | {what} |")
    from tritondl.utils.metrics import HELP
    out += ["", "## Metrics (`TRITONDL_METRICS_ADDR` / `--metrics-addr`: `/metrics`, `/healthz`)", "",
            "Prometheus text format, prefix `tritondl_`; the pool (`python -m tritondl.parallel",
            "--health-addr`) serves the `pool_*` families.", "", "| family | meaning |", "|---|---|"]
    for name, what in sorted(HELP.items()):
        out.append(f"| `tritondl_{name}` | {what} |")
    out += ["", "## Benchmark and test harness only", "", "| variable | effect |", "|---|---|"]
    for var, what in sorted(HARNESS.items()):
        out.append(f"| `{var}` | {what} |")
    return "\n".join(out) + "\n"


def main() -> int:
    text = render()
    if "--check" in sys.argv:
        try:
            cur = open(OUT).read()
        except OSError:
            cur = ""
        if cur != text:
            print("docs/CONFIG.md is out of date: run python tools/gen_config_doc.py", file=sys.stderr)
            return 1
        return 0
    with open(OUT, "w") as f:
        f.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
