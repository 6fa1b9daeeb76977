"""Spare-file recycling for the download directory (``--cleanup`` only).

With cleanup on, every finished job's dir is deleted.  Deleting a 10 MiB file
makes the kernel free its 2,560 page-cache pages (and the filesystem its
blocks), and the next job's download allocates as many again: on the box
that is ~0.25 ms for the unlink plus ~0.7 ms of page allocation inside the
receive pump's pwrites, against ~0.3 ms to overwrite pages that are already
there (``tools/cost_probe.py`` ``unlink`` / ``pwrite_new`` / ``pwrite_reuse``).

So the reaper offers a finished job's files (largest first) to a small
per-process pool (``<download_dir>/.tritondl-spare-<pid>/``) instead of
deleting them, and the HTTP downloader, starting a fresh (non-resumed)
``.part`` file, renames a spare into place and resizes it instead of
creating one.  Bytes the new download has not written yet are the previous
job's; nothing reads them:

* the streamed upload only reads ranges the receive pumps have published;
* resume trusts only the segment counts saved in ``.part.meta``;
* the ``.part`` becomes the destination only after every byte arrived.

Torrent storage does not take spares: the 1 GiB pack job measured no
faster with them (``profiles/r03_recycle_bt/``).

The pool is bounded (files, total bytes, bytes per file), lives on the
download filesystem (a rename, never a copy), is deleted on shutdown, and
pools left by dead processes are swept at start-up.  The reference never
deletes anything (B15), so it has no counterpart.
"""

from __future__ import annotations

import os
import shutil
import stat
import threading

PREFIX = ".tritondl-spare-"

_pools: dict[str, "SparePool"] = {}        # download root -> pool
_lock = threading.Lock()


class SparePool:
    def __init__(self, base_dir: str, max_bytes: int = 1 << 30, max_files: int = 4,
                 max_file_bytes: int | None = None, min_file_bytes: int = 1 << 20) -> None:
        self.base_dir = os.path.abspath(base_dir)
        self.root = os.path.join(self.base_dir, f"{PREFIX}{os.getpid()}")
        self.max_bytes, self.max_files = max_bytes, max_files
        self.max_file_bytes = max_bytes if max_file_bytes is None else max_file_bytes
        self.min_file_bytes = min_file_bytes
        self._files: list[tuple[str, int]] = []    # (path, size), most recent last
        self._bytes = 0
        self._seq = 0
        self._mu = threading.Lock()
        self.taken = self.offered = 0

    # ---------------------------------------------------------------- reaper side
    def offer(self, path: str) -> bool:
        """Keep ``path`` (a finished job's file) as a spare if the pool has room;
        the caller deletes it otherwise."""
        try:
            st = os.stat(path, follow_symlinks=False)
        except OSError:
            return False
        size = st.st_size
        if not (stat.S_ISREG(st.st_mode) and self.min_file_bytes <= size <= self.max_file_bytes):
            return False
        with self._mu:
            if len(self._files) >= self.max_files or self._bytes + size > self.max_bytes:
                return False
            self._seq += 1
            dst = os.path.join(self.root, str(self._seq))
            try:
                os.rename(path, dst)
            except OSError:
                return False
            self._files.append((dst, size))
            self._bytes += size
            self.offered += 1
            return True

    def offer_dir(self, path: str) -> int:
        """Offer the regular files under the job dir ``path``, largest first,
        until the pool is full; returns how many it kept."""
        found = []
        for dirpath, _dirs, names in os.walk(path):
            for n in names:
                p = os.path.join(dirpath, n)
                try:
                    s = os.stat(p, follow_symlinks=False)
                except OSError:
                    continue
                if self.min_file_bytes <= s.st_size <= self.max_file_bytes and os.path.isfile(p) \
                        and not os.path.islink(p):
                    found.append((s.st_size, p))
        kept = 0
        for _size, p in sorted(found, reverse=True):
            if not self.offer(p):
                break
            kept += 1
        return kept

    # ---------------------------------------------------------------- downloader side
    def take(self, dst: str) -> bool:
        """Rename the most recent spare (warmest in the page cache) to ``dst``.
        False if the pool is empty or the rename fails; the caller then
        creates the file as usual."""
        with self._mu:
            while self._files:
                path, size = self._files.pop()
                self._bytes -= size
                try:
                    os.rename(path, dst)
                except OSError:
                    continue
                self.taken += 1
                return True
        return False

    def release(self) -> int:
        """Delete every spare (a download needs their disk space); returns
        the bytes freed."""
        with self._mu:
            files, self._files, self._bytes = self._files, [], 0
        for path, _size in files:
            try:
                os.unlink(path)
            except OSError:
                pass
        return sum(size for _p, size in files)

    def clear(self) -> None:
        with self._mu:
            self._files.clear()
            self._bytes = 0
        shutil.rmtree(self.root, ignore_errors=True)


def register(pool: SparePool) -> SparePool:
    """Make ``pool`` the one downloads under ``pool.base_dir`` take from."""
    os.makedirs(pool.root, mode=0o700, exist_ok=True)
    with _lock:
        _pools[pool.base_dir] = pool
    return pool


def unregister(pool: SparePool) -> None:
    with _lock:
        if _pools.get(pool.base_dir) is pool:
            del _pools[pool.base_dir]


def pool_for(path: str) -> SparePool | None:
    """The pool serving a job dir under one of the registered download roots."""
    if not _pools:
        return None
    parent = os.path.dirname(os.path.abspath(path))
    while True:
        p = _pools.get(parent)
        if p is not None:
            return p
        up = os.path.dirname(parent)
        if up == parent:
            return None
        parent = up


def stale_pools(base_dir: str) -> list[str]:
    """Spare dirs under ``base_dir`` left by processes that no longer run."""
    out = []
    try:
        names = os.listdir(base_dir)
    except OSError:
        return out
    for n in names:
        if not n.startswith(PREFIX):
            continue
        try:
            pid = int(n[len(PREFIX):])
        except ValueError:
            continue
        if pid == os.getpid():
            continue
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            out.append(os.path.join(base_dir, n))
        except PermissionError:
            pass                                   # alive, another user's
    return out
