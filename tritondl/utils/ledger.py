"""Node-level records kept in the work dir, shared by every worker whose
``DOWNLOAD_DIR`` is the same (a pool on one node, or workers in separate
containers that mount one volume).

:class:`DoneLedger` remembers which jobs this node finished, so a copy of a
finished job that comes back is acked instead of run again.  Copies come
back when an ack went nowhere (the broker closed the channel for its
``consumer_timeout``, or the connection dropped), when a lease ran out
during a long broker outage, and when another worker handed a duplicate back
because this one was running the job (``X-Busy``).  The reference had no such
record: it held every delivery unacked for its whole job
(``cmd/downloader/downloader.go:103-155``), so a requeued delivery always
ran again.

Job-dir markers (:data:`RUNNING`, :data:`OURS`) say that a dir belongs to
this worker and whether a run in it ended: a dir still marked running after
its lock is free was left by a worker that died mid-job.
"""

from __future__ import annotations

import hashlib
import os
import time

# in a job dir: a run is in progress (created when the job starts; renamed to OURS when the
# run ends, or deleted with the dir).  Left behind, the worker died mid-job
RUNNING = ".tritondl-running"
# in a job dir: made by this worker (the stale-dir janitor only sweeps dirs carrying a marker)
OURS = ".tritondl-job"


def mark_running(job_dir: str) -> None:
    """One ``open(O_CREAT)``: a few microseconds on the job's path."""
    os.close(os.open(os.path.join(job_dir, RUNNING), os.O_WRONLY | os.O_CREAT | os.O_CLOEXEC, 0o644))


def mark_ended(job_dir: str) -> None:
    """The run in ``job_dir`` ended (settled, or cancelled by a shutdown)."""
    try:
        os.replace(os.path.join(job_dir, RUNNING), os.path.join(job_dir, OURS))
    except FileNotFoundError:
        pass


def was_running(job_dir: str) -> bool:
    return os.path.exists(os.path.join(job_dir, RUNNING))


def is_ours(job_dir: str) -> bool:
    return os.path.exists(os.path.join(job_dir, OURS)) or os.path.exists(os.path.join(job_dir, RUNNING))


class DoneLedger:
    """One empty file per finished job under ``<base>/.tritondl-done/``, named
    by the digest of the job's message body; its mtime is when the job
    finished.  Entries older than ``ttl_s`` no longer count and are swept."""

    DIR = ".tritondl-done"

    def __init__(self, base: str, ttl_s: float = 24 * 3600.0) -> None:
        self.dir = os.path.join(base, self.DIR)
        self.ttl_s = ttl_s

    @staticmethod
    def key(body: bytes) -> str:
        return hashlib.sha256(body).hexdigest()[:32]

    def _path(self, body: bytes) -> str:
        return os.path.join(self.dir, self.key(body))

    def add(self, body: bytes) -> None:
        """Record ``body``'s job as finished now (``O_TRUNC`` refreshes the
        mtime of an entry that exists)."""
        p = self._path(body)
        flags = os.O_WRONLY | os.O_CREAT | os.O_TRUNC | os.O_CLOEXEC
        try:
            fd = os.open(p, flags, 0o644)
        except FileNotFoundError:
            os.makedirs(self.dir, exist_ok=True)
            fd = os.open(p, flags, 0o644)
        os.close(fd)

    def has(self, body: bytes, now: float | None = None) -> bool:
        try:
            st = os.stat(self._path(body))
        except OSError:
            return False
        return (time.time() if now is None else now) - st.st_mtime <= self.ttl_s

    def forget(self, body: bytes) -> None:
        try:
            os.unlink(self._path(body))
        except OSError:
            pass

    def sweep(self, now: float | None = None) -> int:
        """Delete entries past the TTL; returns how many."""
        now = time.time() if now is None else now
        n = 0
        try:
            it = os.scandir(self.dir)
        except OSError:
            return 0
        with it:
            for e in it:
                try:
                    if now - e.stat().st_mtime > self.ttl_s:
                        os.unlink(e.path)
                        n += 1
                except OSError:
                    continue
        return n
