"""Free-space preflight for job directories.

The reference let grab / anacrolix write until the disk filled (then the job
failed half-way, after using the space other jobs needed).  Downloads here
check ``statvfs`` once the size is known — the HTTP probe's length, the
torrent's info dict — and fail the job at once with a clear error (it is
retried / dead-lettered like any other failure) instead.
"""

from __future__ import annotations

import os


class DiskSpaceError(OSError):
    pass


def free_bytes(path: str) -> int:
    """Bytes available to this (unprivileged) process on ``path``'s filesystem;
    walks up to the nearest existing directory."""
    p = os.path.abspath(path)
    while not os.path.exists(p):
        parent = os.path.dirname(p)
        if parent == p:
            break
        p = parent
    st = os.statvfs(p)
    return st.f_bavail * st.f_frsize


def check_space(path: str, need: int, reserve: int = 0) -> None:
    """Raise :class:`DiskSpaceError` unless ``need`` more bytes fit on ``path``'s
    filesystem with ``reserve`` bytes left over."""
    if need <= 0:
        return
    free = free_bytes(path)
    if need + max(0, reserve) > free:
        raise DiskSpaceError(f"not enough disk space in {path}: need {need} bytes, "
                             f"{free} free (reserve {max(0, reserve)})")
