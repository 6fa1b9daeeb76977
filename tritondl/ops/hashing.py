"""Python surface of the native hashing layer.

Host module ``tritondl._hash_host`` (C++/OpenSSL) is mandatory: importing
this module fails loudly if it has not been built (``python
tools/build_native.py``) — there is no silent pure-Python fallback.

GPU module ``tritondl._gpu_hash`` (HIP, gfx950) is used for batched piece
verification when a device is present (``device="auto"``) or demanded
(``device="gpu"``: raises if unavailable).  ``device="hybrid"`` runs the GPU
pipeline and the host's SHA-NI threads on the same layout at once, from
opposite ends (the GPU path is bound by host->HBM staging, not the kernel,
so the idle CPU cores add throughput instead of waiting).
"""

from __future__ import annotations

import os
import sys
import threading
from typing import Sequence

try:
    from .. import _hash_host as _host  # type: ignore[attr-defined]
except ImportError as e:  # pragma: no cover - exercised only on broken builds
    raise ImportError("tritondl native host hashing extension is not built; run "
                      "`python tools/build_native.py` (or __graft_entry__.build())") from e

DIGEST_LEN = {"sha1": 20, "sha256": 32, "md5": 16}

Hasher = _host.Hasher


def digest(kind: str, data) -> bytes:
    return _host.digest(kind, data)


def hash_file(path: str, kinds: Sequence[str] = ("sha256",), offset: int = 0, length: int = -1,
              bufsize: int = 1 << 20) -> dict:
    """One pass over (part of) a file computing several digests; adds ``size``."""
    return _host.hash_file(path, list(kinds), offset, length, bufsize)


def hmac_sha256(key: bytes, msg: bytes) -> bytes:
    return _host.hmac_sha256(key, msg)


def sha_mb() -> bool:
    """Groups of 16 equal-length SHA-1/SHA-256 messages run on the host's
    16-lane AVX-512 kernels (csrc/hash/sha1_mb.h, sha256_mb.h)."""
    return bool(getattr(_host, "sha_mb", lambda: False)())


def chunk_signatures(signing_key: bytes, amzdate: str, scope: str, seed_signature: str, data,
                     chunk_size: int, include_final: bool = True, threads: int = 1) -> list[str]:
    """aws-chunked signature chain over ``data`` (one per ``chunk_size`` chunk,
    plus the terminating empty chunk when ``include_final``).  The per-chunk
    SHA-256 map runs on ``threads`` threads (0 = all); the HMAC chain is serial."""
    return _host.chunk_signatures(signing_key, amzdate, scope, seed_signature, data, chunk_size, include_final,
                                  threads)


def aws_chunk_encode(signing_key: bytes, amzdate: str, scope: str, prev_signature: str, data, chunk_size: int,
                     final: bool = False, threads: int = 1) -> tuple[bytes, str]:
    """Fused aws-chunked framing + signature chain; returns (encoded, last_signature).
    Hash+copy is a parallel map over chunks (``threads``), the chain a serial scan."""
    return _host.aws_chunk_encode(signing_key, amzdate, scope, prev_signature, data, chunk_size, final, threads)


def aws_chunk_decode(signing_key: bytes, amzdate: str, scope: str, seed_signature: str, raw, threads: int = 1,
                     want_data: bool = True, require_final: bool = True) -> tuple[bool, bytes | None, str]:
    """Verify every chunk signature of an aws-chunked body (or, with
    ``require_final=False``, a run of whole frames) and decode it."""
    return _host.aws_chunk_decode(signing_key, amzdate, scope, seed_signature, raw, threads, want_data,
                                  require_final)


# ----------------------------------------------------------------- GPU

_gpu_mod = None
_gpu_lock = threading.Lock()
_gpu_hashers: dict[tuple, object] = {}


def _torch_hip_runtime() -> str | None:
    """Path of the HIP runtime torch ships (``torch/lib/libamdhip64.so``),
    found without importing torch."""
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.origin:
        return None
    p = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    return p if os.path.exists(p) else None


def _load_gpu():
    global _gpu_mod
    if _gpu_mod is None:
        # One HIP runtime per process.  torch ships its own libamdhip64 (SONAME
        # libamdhip64.so.7, loaded by path from torch/lib); if our extension
        # were loaded first its DT_NEEDED would bind ROCm's copy, and a later
        # ``import torch`` would bring up a second HSA runtime that fights over
        # the device ("No HIP GPUs are available").  So map torch's runtime
        # first — by dlopen, not by importing torch: the worker needs only the
        # HIP runtime, and ``import torch`` cost ~1.2 GB of RSS and a 1-2 s GIL
        # stall per worker.  The extension's DT_NEEDED then binds
        # to the already-loaded SONAME.  Without torch installed, ROCm's own.
        if "torch" not in sys.modules:
            hip = _torch_hip_runtime()
            if hip is not None:
                import ctypes
                try:
                    ctypes.CDLL(hip, mode=ctypes.RTLD_GLOBAL)
                except OSError:
                    pass
        from .. import _gpu_hash  # type: ignore[attr-defined]
        _gpu_mod = _gpu_hash
    return _gpu_mod


def gpu_module():
    """Return the HIP extension module (raises ImportError if not built)."""
    return _load_gpu()


def helper_mode() -> bool:
    """GPU verification runs in a helper process (``ops/gpu_helper.py``) so
    the worker never brings up HIP (~850 MB of RSS it could not give back);
    ``TRITONDL_GPU_HELPER=0`` runs it in-process.  The helper itself, tests
    and benches that call :func:`gpu_hasher` directly are in-process."""
    from .gpu_helper import CHILD_ENV
    return os.environ.get("TRITONDL_GPU_HELPER", "1")[:1] not in ("0", "n", "o") and \
        os.environ.get(CHILD_ENV) != "1"


def _kfd_gpus() -> int:
    """GPUs the kernel driver exposes (KFD topology nodes with a gpu_id),
    minus what the visibility variables hide — without touching HIP."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() not in ("", "-1")]
            if not ids:
                return 0
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(base):
            try:
                with open(os.path.join(base, node, "gpu_id")) as f:
                    n += int(f.read().strip() or 0) != 0
            except (OSError, ValueError):
                continue
    except OSError:
        return 0
    return n if os.access("/dev/kfd", os.R_OK | os.W_OK) else 0


def _gpu_ext_present() -> bool:
    import importlib.util
    try:
        return importlib.util.find_spec("tritondl._gpu_hash") is not None
    except (ImportError, ValueError):
        return False


_gpu_disabled: str | None = None
_gpu_disabled_until = 0.0          # monotonic time the GPU is offered again
_gpu_failures = 0                  # consecutive failed GPU calls
GPU_MAX_FAILURES = 3               # consecutive failures before the GPU is set aside
GPU_COOLDOWN_S_DEFAULT = 600.0     # TRITONDL_GPU_COOLDOWN_S


def disable_gpu(reason: str, cooldown: float | None = None) -> None:
    """Stop offering the GPU to ``device="auto"`` callers in this process for
    ``cooldown`` seconds (default ``TRITONDL_GPU_COOLDOWN_S``, 600): a broken
    HIP stack must not fail every resume, and a transient fault (a driver
    reset, one slow call) must not cost the worker its GPU for good."""
    global _gpu_disabled, _gpu_disabled_until
    import time
    if cooldown is None:
        cooldown = float(os.environ.get("TRITONDL_GPU_COOLDOWN_S", "") or GPU_COOLDOWN_S_DEFAULT)
    if _gpu_disabled is None:
        from ..utils.log import log
        log.with_fields(reason=reason, retry_in_s=cooldown).warn("GPU verification set aside; hashing on the host")
    _gpu_disabled = reason
    _gpu_disabled_until = time.monotonic() + cooldown


def note_gpu_failure(reason: str, *, fatal: bool = False) -> bool:
    """A GPU call failed (the helper died, made no progress, or could not
    start).  The GPU is set aside after :data:`GPU_MAX_FAILURES` consecutive
    failures, or at once when ``fatal`` (the helper cannot start).  True if
    it was set aside."""
    global _gpu_failures
    _gpu_failures += 1
    if fatal or _gpu_failures >= GPU_MAX_FAILURES:
        disable_gpu(reason)
        return True
    from ..utils.log import log
    log.with_fields(reason=reason, failures=_gpu_failures).warn("GPU call failed; this batch hashes on the host")
    return False


def note_gpu_success() -> None:
    global _gpu_failures
    _gpu_failures = 0


def _gpu_set_aside() -> bool:
    """True while the GPU is set aside; clears it once the cool-down is over."""
    global _gpu_disabled, _gpu_failures
    if _gpu_disabled is None:
        return False
    import time
    if time.monotonic() < _gpu_disabled_until:
        return True
    from ..utils.log import log
    log.with_field("after", _gpu_disabled).info("offering the GPU for verification again")
    _gpu_disabled = None
    _gpu_failures = 0
    return False


def gpu_available() -> bool:
    if os.environ.get("TRITONDL_GPU_VERIFY", "").lower() == "off" or _gpu_set_aside():
        return False
    if helper_mode():
        return _gpu_ext_present() and _kfd_gpus() > 0
    try:
        return _load_gpu().device_count() > 0
    except Exception:
        return False


_helper = None


def __getattr__(name: str):
    if name == "HelperError":            # lazily: gpu_helper imports this module
        from .gpu_helper import HelperError
        return HelperError
    raise AttributeError(name)


def gpu_backend():
    """What the verification paths hash on: the helper process's hasher
    (default), or the in-process :func:`gpu_hasher`."""
    global _helper
    if not helper_mode():
        return gpu_hasher()
    with _gpu_lock:
        if _helper is None:
            from .gpu_helper import GpuHelper
            _helper = GpuHelper()
        return _helper


def default_device() -> int:
    """This worker's GPU: ``TRITONDL_GPU_DEVICE``, else torchrun's ``LOCAL_RANK``
    (one worker per GPU), modulo the visible devices.  The supervised pool
    (``parallel/pool.py``) pins each worker with ``HIP_VISIBLE_DEVICES``, so
    there it is always 0."""
    want = os.environ.get("TRITONDL_GPU_DEVICE") or os.environ.get("LOCAL_RANK") or "0"
    try:
        n = _load_gpu().device_count()
    except Exception:  # noqa: BLE001 - no extension / no device: callers fail later, loudly
        return 0
    return int(want) % n if n > 0 else 0


def _env_bytes(name: str, default: int) -> int:
    """``123``, ``64M``, ``8G`` (binary units)."""
    v = os.environ.get(name, "").strip().upper()
    if not v:
        return default
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30, "T": 1 << 40}.get(v[-1:], 1)
    return int(float(v[:-1] if mult > 1 else v) * mult)


GPU_MAX_HBM_DEFAULT = 8 << 30     # the two HBM windows together (TRITONDL_GPU_MAX_HBM)
GPU_IDLE_S_DEFAULT = 30.0         # free windows + pinned staging after this long unused (TRITONDL_GPU_IDLE_S)


def gpu_hasher(device: int | None = None, batch_bytes: int = 0, reader_threads: int = 0, window_bytes: int = 0):
    """Cached per-device :class:`GpuHasher`.  ``batch_bytes`` is the pinned
    staging slot, one of a ring of 4 (0: ``TRITONDL_GPU_STAGE_MB`` or 128 MiB); ``reader_threads``
    the pread threads filling it (0: ``TRITONDL_GPU_READERS`` or
    :data:`GPU_READERS`); ``window_bytes`` the HBM window hashed per kernel
    launch (0 = auto: half of ``TRITONDL_GPU_MAX_HBM`` (default 8 GiB), at
    most a third of free HBM).  Nothing is allocated until a call needs it,
    and everything is freed again after ``TRITONDL_GPU_IDLE_S`` (default 30 s)
    without a call: an idle ingest worker holds no HBM and no pinned memory."""
    device = default_device() if device is None else device
    batch_bytes = batch_bytes or (int(os.environ.get("TRITONDL_GPU_STAGE_MB", "128")) << 20)
    reader_threads = reader_threads or int(os.environ.get("TRITONDL_GPU_READERS", str(GPU_READERS)))
    max_hbm = _env_bytes("TRITONDL_GPU_MAX_HBM", GPU_MAX_HBM_DEFAULT)
    key = (device, max(batch_bytes, 1 << 20), window_bytes, reader_threads, max_hbm)
    with _gpu_lock:
        h = _gpu_hashers.get(key)
        if h is None:
            h = _load_gpu().GpuHasher(device, batch_bytes, reader_threads, window_bytes, max_hbm)
            h.trace = os.environ.get("TRITONDL_GPU_TRACE", "") == "1"
            _gpu_hashers[key] = h
            _start_idle_reaper()
        return h


_reaper: threading.Thread | None = None


def gpu_idle_seconds() -> float:
    return float(os.environ.get("TRITONDL_GPU_IDLE_S", GPU_IDLE_S_DEFAULT))


def release_idle_gpu(idle_s: float | None = None) -> int:
    """Free the buffers of every hasher unused for ``idle_s`` seconds; returns
    how many were released (the idle reaper's one step; tests call it)."""
    idle = gpu_idle_seconds() if idle_s is None else idle_s
    with _gpu_lock:
        hs = list(_gpu_hashers.values())
    return sum(1 for h in hs if h.release_if_idle(idle))


def _start_idle_reaper() -> None:
    """One daemon thread per process (caller holds _gpu_lock)."""
    global _reaper
    if _reaper is not None:
        return

    def loop() -> None:
        import time
        while True:
            idle = gpu_idle_seconds()                 # re-read: <= 0 turns the reaper off
            time.sleep(max(0.05, min(5.0, idle / 3)) if idle > 0 else 5.0)
            if idle <= 0:
                continue
            try:
                release_idle_gpu(idle)
            except Exception:  # noqa: BLE001 - never let the reaper die; the next step retries
                pass
    _reaper = threading.Thread(target=loop, name="tdl-gpu-idle", daemon=True)
    _reaper.start()


def warm_gpu(device: int | None = None) -> bool:
    """Bring up the HIP context and load the code object (one tiny batch) so
    the first resume-verify of a job does not pay the one-time setup, then
    free the batch's buffers again: warm-up leaves no HBM or pinned memory
    allocated.  In helper mode nothing is started unless
    ``TRITONDL_GPU_WARMUP=1`` (the helper would exit idle again anyway).
    Returns False when no GPU path is available."""
    if not gpu_available():
        return False
    if helper_mode():
        if os.environ.get("TRITONDL_GPU_WARMUP", "") == "1":
            gpu_backend().hash_buffer("sha1", b"\0" * 16384, 16384)
        return True
    h = gpu_hasher(device)
    h.hash_buffer("sha1", b"\0" * 16384, 16384)
    h.release()
    return True


DEVICES = ("auto", "cpu", "gpu", "hybrid")
GPU_READERS = 8            # pread threads feeding the GPU's pinned staging (gpu_hasher default)


def timeline_summary(tl) -> dict:
    """Overlap of a :attr:`GpuHasher.last_timeline` (``trace`` on): busy time of
    H2D copies and of kernels (interval unions), how much of the kernel time
    ran under copies, and the copy engine's rate while busy."""
    def union(iv):
        out: list[list[float]] = []
        for a, b in sorted(iv):
            if out and a <= out[-1][1]:
                out[-1][1] = max(out[-1][1], b)
            else:
                out.append([a, b])
        return out

    def inter(x, y):
        i = j = 0
        tot = 0.0
        while i < len(x) and j < len(y):
            a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
            tot += max(0.0, b - a)
            if x[i][1] < y[j][1]:
                i += 1
            else:
                j += 1
        return tot
    h2d = union([(a, b) for k, a, b, _n in tl if k.startswith("h2d")])        # staged + direct copies
    ker = union([(a, b) for k, a, b, _n in tl if k == "kernel"])
    nbytes = sum(n for k, _a, _b, n in tl if k.startswith("h2d"))
    busy = sum(b - a for a, b in h2d)
    span = max((b for _k, _a, b, _n in tl), default=0.0)
    return {"h2d_ms": round(busy, 3), "h2d_count": sum(1 for x in tl if x[0].startswith("h2d")),
            "h2d_direct_count": sum(1 for x in tl if x[0] == "h2d_direct"),
            "kernel_ms": round(sum(b - a for a, b in ker), 3), "kernels": sum(1 for x in tl if x[0] == "kernel"),
            "kernel_under_h2d_ms": round(inter(ker, h2d), 3), "span_ms": round(span, 3),
            "h2d_GBps_busy": round(nbytes / busy / 1e6, 1) if busy else None}


def _resolve(device: str) -> str:
    if device == "auto":
        return "gpu" if gpu_available() else "cpu"
    if device not in DEVICES:
        raise ValueError(f"device must be one of {'|'.join(DEVICES)}, got {device!r}")
    if device in ("gpu", "hybrid") and not gpu_available():
        raise RuntimeError(f"{device} hashing requested but no HIP device / _gpu_hash extension available")
    return device


def gpu_direct() -> bool:
    """Resident file data is DMA'd to HBM straight from the page cache
    (registered read-only mappings, no reader threads); ``TRITONDL_GPU_DIRECT=0``
    sends everything through the pinned staging ring."""
    return os.environ.get("TRITONDL_GPU_DIRECT", "1")[:1] not in ("0", "n", "o")


def hybrid_cpu_threads(cpus: int | None = None) -> int:
    """Host hashing threads that work next to the GPU pipeline
    (``TRITONDL_HYBRID_CPU_THREADS`` overrides): every CPU but the one driving
    the GPU when its copies come straight from the page cache, else the CPUs
    left by the staging readers."""
    env = os.environ.get("TRITONDL_HYBRID_CPU_THREADS")
    if env:
        return max(1, int(env))
    n = cpus or effective_cpus()
    if gpu_direct():
        return max(1, n - 1)
    return max(1, n - int(os.environ.get("TRITONDL_GPU_READERS", str(GPU_READERS))))


# Cost model for device="auto" batch verification, calibrated on MI355X with
# the box's 16-CPU share (profiles/r01_hash_v3_windows, profiles/r02_sha1_ab):
# the GPU path is bounded by host->HBM copies (~45 GB/s) plus, because the
# kernel runs one lane per piece, the per-lane SHA-1 rate (~55 MB/s) for one
# piece; the host path runs ~1.5 GB/s per thread through OpenSSL, ~3 GB/s
# with the two-stream SHA-NI pairs (8 GiB v1 resume on 16 threads: 35 -> 55
# GB/s), ~4.4 GB/s with the 16-lane AVX-512 SHA-1 (70 GB/s on 16 threads,
# profiles/r03_sha1_mb), plus ~15 us of per-piece overhead.
GPU_COPY_BPS = 55e9 if gpu_direct() else 45e9   # direct from the page cache: 57.6 GB/s (profiles/r03_reg_probe)
GPU_LANE_BPS = 55e6
GPU_SETUP_S = 5e-3
CPU_THREAD_BPS = (4.4e9 if sha_mb() else
                  3.0e9 if getattr(_host, "sha_ni", lambda: False)() else 1.5e9)
CPU_PIECE_S = 15e-6


def effective_cpus() -> int:
    """CPUs this process may actually use: affinity mask and cgroup v2 quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def choose_device(n_pieces: int, piece_len: int, total: int, cpu_threads: int | None = None,
                  lane_len: int | None = None) -> str:
    """cpu | gpu | hybrid for a batch verify, by the cost model above.  In
    hybrid mode the CPU threads left next to the GPU readers add their rate
    to the GPU's (the native claim rule also hands the GPU's last-kernel
    latency tail to the CPU, so hybrid is never slower than its GPU part).
    ``lane_len``: bytes one GPU lane hashes serially (default ``piece_len``;
    16 KiB for BEP 52 merkle leaves, where the host still reads whole
    pieces, so its per-piece overhead counts ``n_pieces`` pieces)."""
    if n_pieces == 0 or not gpu_available():
        return "cpu"
    lane = lane_len or piece_len
    cpus = cpu_threads or effective_cpus()
    thr = max(1, min(cpus, n_pieces))
    t_gpu = total / GPU_COPY_BPS + lane / GPU_LANE_BPS + GPU_SETUP_S
    t_cpu = (total / CPU_THREAD_BPS + n_pieces * CPU_PIECE_S) / thr
    hthr = hybrid_cpu_threads(cpus)
    cpu_bps = hthr * CPU_THREAD_BPS / (1 + CPU_PIECE_S * CPU_THREAD_BPS / piece_len)
    t_hyb = max(total / (GPU_COPY_BPS + cpu_bps), lane / GPU_LANE_BPS) + GPU_SETUP_S
    best = min(t_cpu, t_gpu, t_hyb)
    if best == t_cpu:
        return "cpu"
    return "hybrid" if best == t_hyb and hthr >= 2 else "gpu"


def piece_hashes(data, piece_len: int, kind: str = "sha1", device: str = "cpu", threads: int = 0) -> bytes:
    """Concatenated digests of ``data`` split into ``piece_len`` pieces."""
    dev = _resolve(device)
    if dev == "gpu":
        return gpu_backend().hash_buffer(kind, data, piece_len)
    return _host.piece_hashes(kind, data, piece_len, threads or effective_cpus())


def merkle_root(data, width: int) -> bytes:
    """BEP 52 root of one piece's data over a ``width``-leaf tree, native
    (SHA-NI pairs, GIL released); ``fetch.bt.merkle.piece_root`` is the spec."""
    return _host.merkle_root(data, width)


def verify_buffers(kind: str, buffers: Sequence, expected: bytes, threads: int = 0) -> bytes:
    """Verify in-memory pieces (any buffer objects) against concatenated
    digests on the host: SHA-NI pairs on ``threads`` threads, GIL released.
    One byte (0/1) per buffer."""
    return _host.verify_buffers(kind, list(buffers), expected, threads)


def verify_pieces(files: Sequence[tuple[str, int]], piece_len: int, expected: bytes, kind: str = "sha1",
                  device: str = "cpu", threads: int = 0) -> bytes:
    """Verify the torrent layout ``files`` [(path, length), ...] against
    ``expected`` (concatenated digests).  Returns one byte (0/1) per piece."""
    dev = _resolve(device)
    files = [(str(p), int(n)) for p, n in files]
    if dev == "gpu":
        return gpu_backend().verify_files(files, piece_len, expected, kind)
    if dev == "hybrid":
        return gpu_backend().verify_files(files, piece_len, expected, kind,
                                          cpu_threads=threads or hybrid_cpu_threads())
    return _host.verify_pieces(files, piece_len, expected, threads or effective_cpus(), kind)


def verify_pieces_v2(files: Sequence[tuple[str, int]], piece_len: int, expected: bytes, widths: Sequence[int],
                     reals: Sequence[int], known: Sequence[bool] | None = None, device: str = "cpu",
                     threads: int = 0) -> bytes:
    """BitTorrent v2 (BEP 52) verification of a piece-aligned layout: piece p's
    16 KiB-leaf merkle root (``widths[p]`` leaves, ``reals[p]`` data bytes)
    must equal ``expected[32p:32p+32]``.  Host: threaded read+hash+reduce per
    piece.  GPU: the HIP kernel hashes every 16 KiB leaf of the layout (the
    lane-parallel case it is fastest at), the host reduces the small trees."""
    dev = _resolve(device)
    files = [(str(p), int(n)) for p, n in files]
    n = len(widths)
    kn = bytes(1 if k else 0 for k in (known if known is not None else [True] * n))
    thr = threads or effective_cpus()
    if dev in ("gpu", "hybrid"):
        leaves, leaf_ok = gpu_backend().digest_files(files, 16384, "sha256",
                                                     cpu_threads=hybrid_cpu_threads() if dev == "hybrid" else 0)
        leaves, leaf_ok = bytearray(leaves), bytearray(leaf_ok)
        # the kernel hashed whole 16 KiB blocks of the padded stream; a file's
        # short last leaf must hash only its real bytes: redo those (<= one per file)
        per = piece_len // 16384
        for p in range(n):
            tail = reals[p] % 16384
            if not kn[p] or not tail:
                continue
            k = p * per + reals[p] // 16384
            data = _read_layout(files, p * piece_len + reals[p] - tail, tail)
            if data is None:
                leaf_ok[k] = 0
            else:
                leaves[32 * k:32 * k + 32] = _host.digest("sha256", data)
        return _host.merkle_check(bytes(leaves), bytes(leaf_ok), piece_len, expected, list(widths), list(reals),
                                  kn, thr)
    return _host.merkle_verify(files, piece_len, expected, list(widths), list(reals), kn, thr)


def _read_layout(files: Sequence[tuple[str, int]], off: int, n: int) -> bytes | None:
    """``n`` bytes at stream offset ``off`` of a file layout ("" = zeros)."""
    out = bytearray()
    pos = 0
    for path, ln in files:
        a, b = max(off, pos), min(off + n, pos + ln)
        if a < b:
            if not path:
                out += bytes(b - a)
            else:
                try:
                    fd = os.open(path, os.O_RDONLY)
                except OSError:
                    return None
                try:
                    chunk = os.pread(fd, b - a, a - pos)
                finally:
                    os.close(fd)
                if len(chunk) != b - a:
                    return None
                out += chunk
        pos += ln
        if pos >= off + n:
            break
    return bytes(out) if len(out) == n else None
