"""GPU piece verification in a helper process that lives only while it is used.

Bringing up the HIP runtime costs a process ~850 MB of resident memory
(measured on the MI355X box, ``profiles/r04_rss/``: ~600 MB at the first HIP
call, the rest with the first kernel and pinned staging) and it cannot be
given back short of exiting.  An ingest worker verifies torrent pieces on the
GPU only when a job resumes (the reference has no GPU state at all), so the
worker never initialises HIP itself: the first GPU verification starts this
helper, which owns the :class:`GpuHasher` (HBM windows, pinned staging, the
HIP context), and the helper exits after ``TRITONDL_GPU_IDLE_S`` (30 s)
without a request — returning its host memory, its HBM and its context.
The next resume starts a new one.

The helper reads the torrent files itself (paths travel, not data), so the
pipe carries only the expected digests in and a byte per piece out.

Protocol (stdin/stdout of the helper, binary): a request is one JSON line
``{"op": ..., ..., "blob": n}`` followed by ``n`` raw bytes; a reply is one
JSON line ``{"ok": true, "blob": n, ...}`` (or ``{"error": ...}``) followed
by ``n`` bytes.  The first line the helper writes is ``{"ready": true,
"devices": n}``.

    python -m tritondl.ops.gpu_helper        # spawned by GpuHelper, never by hand
"""

from __future__ import annotations

import json
import os
import select
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD_ENV = "TRITONDL_GPU_HELPER_CHILD"


class HelperError(RuntimeError):
    pass


def _read_exact(f, n: int) -> bytes:
    out = bytearray()
    while len(out) < n:
        b = f.read(n - len(out))
        if not b:
            raise EOFError("helper pipe closed")
        out += b
    return bytes(out)


# ----------------------------------------------------------------- helper side
def _backend():
    """The helper's hasher: the HIP GpuHasher, or (``TRITONDL_GPU_HELPER_FAKE=1``,
    CPU tests of the protocol) a host stand-in with the same methods."""
    from . import hashing
    if os.environ.get("TRITONDL_GPU_HELPER_FAKE") == "1":
        class _Host:
            last_gpu_pieces = 0
            last_direct_bytes = 0
            last_window_bytes = 0

            def verify_files(self, files, piece_len, expected, kind="sha1", cpu_threads=0):
                return hashing._host.verify_pieces(files, piece_len, expected, hashing.effective_cpus(), kind)

            def digest_files(self, files, piece_len, kind="sha256", cpu_threads=0):
                from .hashing import _read_layout
                total = sum(n for _p, n in files)
                data = _read_layout(files, 0, total) or b""
                return hashing._host.piece_hashes(kind, data, piece_len, 1), b"\x01" * (-(-total // piece_len))

            def hash_buffer(self, kind, data, piece_len):
                return hashing._host.piece_hashes(kind, data, piece_len, 1)
        return _Host(), 1
    if not hashing.gpu_available():
        raise HelperError("no HIP device / _gpu_hash extension in the helper")
    return hashing.gpu_hasher(), hashing.gpu_module().device_count()


def serve() -> int:
    """Answer requests until stdin closes or nothing arrives for the idle timeout."""
    from . import hashing
    inp, out = sys.stdin.buffer, sys.stdout.buffer
    try:
        h, ndev = _backend()
    except Exception as e:  # noqa: BLE001 - reported to the client, which fails the call loudly
        out.write((json.dumps({"ready": False, "error": str(e)}) + "\n").encode())
        out.flush()
        return 1
    out.write((json.dumps({"ready": True, "devices": ndev, "pid": os.getpid()}) + "\n").encode())
    out.flush()
    while True:
        idle = hashing.gpu_idle_seconds()
        r, _w, _x = select.select([inp], [], [], idle if idle > 0 else None)
        if not r:
            return 0                                          # idle: exit, freeing HIP, HBM and pinned memory
        line = inp.readline()
        if not line:
            return 0
        try:
            req = json.loads(line)
            blob = _read_exact(inp, int(req.get("blob", 0)))
            rep, data = _dispatch(h, req, blob)
        except EOFError:
            return 0
        except Exception as e:  # noqa: BLE001 - one bad request must not kill the helper
            rep, data = {"error": f"{type(e).__name__}: {e}"}, b""
        rep["blob"] = len(data)
        out.write((json.dumps(rep) + "\n").encode())
        out.write(data)
        out.flush()


def _dispatch(h, req: dict, blob: bytes) -> tuple[dict, bytes]:
    op = req["op"]
    files = [(str(p), int(n)) for p, n in req.get("files", [])]
    stats = {}
    if op == "ping":
        return {"ok": True}, b""
    stall = float(os.environ.get("TRITONDL_GPU_HELPER_FAKE_STALL", "0") or 0)
    if stall > 0 and os.environ.get("TRITONDL_GPU_HELPER_FAKE") == "1":
        time.sleep(stall)                                   # tests: a helper stuck in a call
    if op == "verify_files":
        data = h.verify_files(files, int(req["piece_len"]), blob, req.get("kind", "sha1"),
                              cpu_threads=int(req.get("cpu_threads", 0)))
    elif op == "digest_files":
        d, ok = h.digest_files(files, int(req["piece_len"]), req.get("kind", "sha256"),
                               cpu_threads=int(req.get("cpu_threads", 0)))
        stats["split"] = len(d)
        data = bytes(d) + bytes(ok)
    elif op == "hash_buffer":
        data = h.hash_buffer(req.get("kind", "sha1"), blob, int(req["piece_len"]))
    else:
        raise ValueError(f"unknown op {op!r}")
    for k in ("last_gpu_pieces", "last_direct_bytes", "last_window_bytes"):
        stats[k] = int(getattr(h, k, 0))
    return {"ok": True, **stats}, bytes(data)


# ----------------------------------------------------------------- worker side
class GpuHelper:
    """The worker's handle on the helper: same verify / digest / hash calls as
    :class:`GpuHasher`, run in the helper, which is started on first use and
    again after it exits idle.  One request at a time (callers are executor
    threads)."""

    def __init__(self, start_timeout: float = 120.0, call_timeout: float | None = None) -> None:
        """``call_timeout``: seconds a call may take before the helper is
        killed and the call fails (:class:`HelperError`, which the "auto"
        verify paths answer by hashing on the host), plus one second per
        256 MB the call hashes.  Default ``TRITONDL_GPU_CALL_TIMEOUT`` (120):
        a helper stuck in the GPU must not pin the worker's executor thread,
        and the job slot with it, forever."""
        self.start_timeout = start_timeout
        self.call_timeout = (float(os.environ.get("TRITONDL_GPU_CALL_TIMEOUT", "120") or 120)
                             if call_timeout is None else call_timeout)
        self._p: subprocess.Popen | None = None
        self._lock = threading.Lock()
        self.spawned = 0
        self.last_gpu_pieces = 0
        self.last_direct_bytes = 0
        self.last_window_bytes = 0

    @property
    def pid(self) -> int | None:
        p = self._p
        return p.pid if p is not None and p.poll() is None else None

    def _spawn(self) -> None:
        env = dict(os.environ)
        env[CHILD_ENV] = "1"
        env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        p = subprocess.Popen([sys.executable, "-m", "tritondl.ops.gpu_helper"], stdin=subprocess.PIPE,
                             stdout=subprocess.PIPE, cwd=ROOT, env=env)
        assert p.stdout is not None
        r, _w, _x = select.select([p.stdout], [], [], self.start_timeout)
        line = p.stdout.readline() if r else b""
        try:
            hello = json.loads(line) if line else {}
        except ValueError:
            hello = {}
        if not hello.get("ready"):
            self._reap(p, kill=True)
            raise HelperError(f"GPU helper failed to start: {hello.get('error') or 'no answer'}")
        self._p = p
        self.spawned += 1

    @staticmethod
    def _reap(p: subprocess.Popen, kill: bool = False) -> int | None:
        try:
            if p.stdin is not None:
                p.stdin.close()
        except OSError:
            pass
        if kill and p.poll() is None:
            p.kill()                                # our own child, by PID
        try:
            return p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            return p.wait()

    def _call(self, req: dict, blob: bytes = b"") -> tuple[dict, bytes]:
        with self._lock:
            for attempt in (0, 1):
                if self._p is None or self._p.poll() is not None:
                    if self._p is not None:
                        self._reap(self._p)
                    self._spawn()
                p = self._p
                assert p is not None and p.stdin is not None and p.stdout is not None
                work = len(blob) + sum(int(n) for _p, n in req.get("files", []))
                limit = self.call_timeout + work / 256e6
                try:
                    p.stdin.write((json.dumps({**req, "blob": len(blob)}) + "\n").encode())
                    p.stdin.write(blob)
                    p.stdin.flush()
                    # one request at a time, so nothing of a later reply can sit in stdout's buffer
                    if not select.select([p.stdout], [], [], limit)[0]:
                        self._reap(p, kill=True)
                        self._p = None
                        raise HelperError(f"GPU helper did not answer {req.get('op')!r} within {limit:.0f}s; "
                                          "killed it")
                    line = p.stdout.readline()
                    if not line:
                        raise EOFError("helper closed its pipe")
                    rep = json.loads(line)
                    data = _read_exact(p.stdout, int(rep.get("blob", 0)))
                except (BrokenPipeError, EOFError, OSError, ValueError) as e:
                    rc = self._reap(p, kill=True)
                    self._p = None
                    # it exited idle just as the request went out: start a new one, once
                    if attempt == 0 and rc == 0:
                        continue
                    raise HelperError(f"GPU helper died (rc={rc}): {e}") from e
                if "error" in rep:
                    raise HelperError(rep["error"])
                for k in ("last_gpu_pieces", "last_direct_bytes", "last_window_bytes"):
                    if k in rep:
                        setattr(self, k, rep[k])
                return rep, data
        raise HelperError("unreachable")

    # GpuHasher-compatible surface
    def verify_files(self, files, piece_len: int, expected: bytes, kind: str = "sha1", cpu_threads: int = 0) -> bytes:
        return self._call({"op": "verify_files", "files": [[str(p), int(n)] for p, n in files],
                           "piece_len": piece_len, "kind": kind, "cpu_threads": cpu_threads}, bytes(expected))[1]

    def digest_files(self, files, piece_len: int, kind: str = "sha256", cpu_threads: int = 0) -> tuple[bytes, bytes]:
        rep, data = self._call({"op": "digest_files", "files": [[str(p), int(n)] for p, n in files],
                                "piece_len": piece_len, "kind": kind, "cpu_threads": cpu_threads})
        k = int(rep["split"])
        return data[:k], data[k:]

    def hash_buffer(self, kind: str, data, piece_len: int) -> bytes:
        return self._call({"op": "hash_buffer", "kind": kind, "piece_len": piece_len}, bytes(data))[1]

    def ping(self) -> bool:
        return bool(self._call({"op": "ping"})[0].get("ok"))

    def close(self) -> None:
        with self._lock:
            if self._p is not None:
                self._reap(self._p)
                self._p = None

    def wait_exit(self, timeout: float) -> bool:
        """Wait for the helper to exit by itself (idle); True once it has."""
        t0 = time.monotonic()
        while time.monotonic() - t0 < timeout:
            p = self._p
            if p is None or p.poll() is not None:
                return True
            time.sleep(0.05)
        return False


def main() -> int:
    return serve()


if __name__ == "__main__":
    sys.exit(main())
