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
by ``n`` bytes.  While a call runs the helper writes a heartbeat line
``{"progress": bytes}`` every second (bytes read since the call began, from
the hasher's lifetime counter): the worker kills the helper only once a
call has made **no progress** for ``TRITONDL_GPU_CALL_TIMEOUT`` seconds, so
a large resume on a slow volume (cold HDD, NFS) is never cut short while it
is still reading.  The first line the helper writes is ``{"ready": true,
"devices": n}``.

A failed call does not turn the GPU off at once: the worker counts
consecutive failures (:func:`tritondl.ops.hashing.note_gpu_failure`) and
stops offering the GPU after ``GPU_MAX_FAILURES`` of them, or at once when
the helper cannot start, and offers it again after
``TRITONDL_GPU_COOLDOWN_S`` (600 s).

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


class HelperStartError(HelperError):
    """The helper process did not come up (no device, a broken HIP stack)."""


def _progress_every() -> float:
    return float(os.environ.get("TRITONDL_GPU_PROGRESS_S", "1") or 1)


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
            read = 0

            def progress(self):
                return self.read

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
            rep, data = _run_with_progress(h, req, blob, out)
        except EOFError:
            return 0
        except Exception as e:  # noqa: BLE001 - one bad request must not kill the helper
            rep, data = {"error": f"{type(e).__name__}: {e}"}, b""
        rep["blob"] = len(data)
        out.write((json.dumps(rep) + "\n").encode())
        out.write(data)
        out.flush()


def _run_with_progress(h, req: dict, blob: bytes, out) -> tuple[dict, bytes]:
    """Run one request on a thread; meanwhile write ``{"progress": n}`` every
    :func:`_progress_every` seconds (bytes the hasher has read since the call
    began).  Writes happen only on this thread, so lines never interleave."""
    if req.get("op") == "ping":
        return _dispatch(h, req, blob)
    res: dict = {}
    base = _progress(h)

    def work() -> None:
        try:
            res["r"] = _dispatch(h, req, blob)
        except BaseException as e:  # noqa: BLE001 - re-raised on the serving thread
            res["e"] = e
    t = threading.Thread(target=work, name="tdl-gpu-call", daemon=True)
    t.start()
    every = _progress_every()
    while True:
        t.join(every)
        if not t.is_alive():
            break
        out.write((json.dumps({"progress": _progress(h) - base}) + "\n").encode())
        out.flush()
    if "e" in res:
        raise res["e"]
    return res["r"]


def _progress(h) -> int:
    try:
        return int(h.progress())
    except Exception:  # noqa: BLE001 - a hasher without the counter: heartbeats carry 0
        return 0


def _dispatch(h, req: dict, blob: bytes) -> tuple[dict, bytes]:
    op = req["op"]
    files = [(str(p), int(n)) for p, n in req.get("files", [])]
    stats = {}
    if op == "ping":
        return {"ok": True}, b""
    if os.environ.get("TRITONDL_GPU_HELPER_FAKE") == "1":
        stall = float(os.environ.get("TRITONDL_GPU_HELPER_FAKE_STALL", "0") or 0)
        if stall > 0:
            time.sleep(stall)                               # tests: a helper stuck in a call (no progress)
        slow = float(os.environ.get("TRITONDL_GPU_HELPER_FAKE_SLOW", "0") or 0)
        t_end = time.monotonic() + slow
        while time.monotonic() < t_end:                     # tests: a slow call that keeps reading
            time.sleep(0.05)
            h.read += 1 << 20
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
        """``call_timeout``: seconds a call may go without progress (no
        heartbeat whose byte count grew) before the helper is killed and the
        call fails (:class:`HelperError`, which the "auto" verify paths answer
        by hashing on the host).  Default ``TRITONDL_GPU_CALL_TIMEOUT`` (120):
        a helper stuck in the GPU must not pin the worker's executor thread,
        and the job slot with it, forever — but a slow volume that is still
        being read is not a stuck helper."""
        self.start_timeout = start_timeout
        self.call_timeout = (float(os.environ.get("TRITONDL_GPU_CALL_TIMEOUT", "120") or 120)
                             if call_timeout is None else call_timeout)
        self._p: subprocess.Popen | None = None
        self._rbuf = bytearray()                 # bytes read from the helper's stdout, not yet consumed
        self._lock = threading.Lock()
        self.spawned = 0
        self.last_beats = 0                      # progress heartbeats received during the last call
        self.last_progress = 0                   # bytes the last heartbeat of the last call reported
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
        self._rbuf.clear()
        try:
            line = self._readline(p, time.monotonic() + self.start_timeout)
            hello = json.loads(line) if line else {}
        except (EOFError, TimeoutError, OSError, ValueError):
            hello = {}
        if not hello.get("ready"):
            self._reap(p, kill=True)
            raise HelperStartError(f"GPU helper failed to start: {hello.get('error') or 'no answer'}")
        self._p = p
        self.spawned += 1

    # The helper's stdout is read with os.read into our own buffer: a reply can
    # follow progress lines in the same read, and select() on the fd cannot see
    # what a buffered reader already holds.
    def _fill(self, p: subprocess.Popen, deadline: float) -> None:
        fd = p.stdout.fileno()  # type: ignore[union-attr]
        left = deadline - time.monotonic()
        if left <= 0 or not select.select([fd], [], [], left)[0]:
            raise TimeoutError
        b = os.read(fd, 1 << 16)
        if not b:
            raise EOFError("helper closed its pipe")
        self._rbuf += b

    def _readline(self, p: subprocess.Popen, deadline: float) -> bytes:
        while True:
            i = self._rbuf.find(b"\n")
            if i >= 0:
                line = bytes(self._rbuf[:i + 1])
                del self._rbuf[:i + 1]
                return line
            self._fill(p, deadline)

    def _read_n(self, p: subprocess.Popen, n: int, deadline: float) -> bytes:
        while len(self._rbuf) < n:
            self._fill(p, deadline)
        data = bytes(self._rbuf[:n])
        del self._rbuf[:n]
        return data

    @staticmethod
    def _reap(p: subprocess.Popen, kill: bool = False) -> int | None:
        """Close the helper's stdin (it exits on EOF) or kill it, and collect it.
        Bounded: a helper stuck in an uninterruptible GPU driver call may not
        die at once after SIGKILL; it is then left to a daemon thread to
        collect, and this returns None, so the caller (holding the call lock)
        never blocks on it."""
        try:
            if p.stdin is not None:
                p.stdin.close()
        except OSError:
            pass
        if kill and p.poll() is None:
            p.kill()                                # our own child, by PID
        try:
            return p.wait(timeout=5 if kill else 30)
        except subprocess.TimeoutExpired:
            p.kill()
        try:
            return p.wait(timeout=5)
        except subprocess.TimeoutExpired:
            threading.Thread(target=p.wait, name="tdl-gpu-reaper", daemon=True).start()
            return None

    def _call(self, req: dict, blob: bytes = b"") -> tuple[dict, bytes]:
        with self._lock:
            for attempt in (0, 1):
                if self._p is None or self._p.poll() is not None:
                    if self._p is not None:
                        self._reap(self._p)
                    self._spawn()
                p = self._p
                assert p is not None and p.stdin is not None and p.stdout is not None
                gap = self.call_timeout
                try:
                    p.stdin.write((json.dumps({**req, "blob": len(blob)}) + "\n").encode())
                    p.stdin.write(blob)
                    p.stdin.flush()
                    # the call may run as long as it keeps making progress: every heartbeat
                    # whose byte count grew pushes the deadline out by `gap`
                    done, deadline = 0, time.monotonic() + gap
                    self.last_beats = self.last_progress = 0
                    while True:
                        try:
                            line = self._readline(p, deadline)
                        except TimeoutError:
                            self._reap(p, kill=True)
                            self._p = None
                            raise HelperError(f"GPU helper did not answer {req.get('op')!r}: no progress for "
                                              f"{gap:.0f}s ({done} bytes read); killed it") from None
                        rep = json.loads(line)
                        if "progress" in rep and "ok" not in rep and "error" not in rep:
                            self.last_beats += 1
                            self.last_progress = int(rep["progress"])
                            if int(rep["progress"]) > done:
                                done = int(rep["progress"])
                                deadline = time.monotonic() + gap
                            continue
                        break
                    data = self._read_n(p, int(rep.get("blob", 0)), time.monotonic() + gap)
                except (BrokenPipeError, EOFError, OSError, ValueError, TimeoutError) as e:
                    rc = self._reap(p, kill=True)
                    self._p = None
                    # it exited idle just as the request went out: start a new one, once
                    if attempt == 0 and rc == 0:
                        continue
                    raise HelperError(f"GPU helper died (rc={rc}): {e}") from e
                if "error" in rep:
                    raise HelperError(rep["error"])
                from . import hashing
                hashing.note_gpu_success()
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
