"""Media-file selector — capability of the reference's ``process.Dir``
(``internal/process/process.go:17-93``, component C8).

Rules:

* top-level entries are read (Lstat semantics); if exactly ONE top-level
  directory exists its name joins the allow-list (``process.go:41-52``);
* the walk is lexical (``filepath.Walk``); the root is always descended and
  every other directory, at any depth, is descended only if its base name
  *contains* an allow-list entry (``"season"`` or the sole TLD) or matches
  ``s\\d+`` anywhere (``process.go:56-72``) — case-sensitive;
* files are kept iff ``filepath.Ext`` is one of ``.mp4 .mkv .mov .webm``;
* the result is a list of cleaned full paths (``[]`` when none); a missing
  root raises.

Deviation (defect B11): the reference dereferences ``info`` before checking
the walk error and panics on an unreadable entry; here the error propagates.
"""

from __future__ import annotations

import os
import re
import stat

from .utils.gocompat import go_base, go_ext, go_join

MEDIA_EXTS = frozenset({".mp4", ".mkv", ".mov", ".webm"})
ALLOWED_DIRS = ("season",)
ALLOWED_DIRS_REGEX = (re.compile(r"s\d+"),)


def _dir_allowed(name: str, allowed: tuple[str, ...]) -> bool:
    for a in allowed:
        if a in name:
            return True
    for rx in ALLOWED_DIRS_REGEX:
        if rx.search(name):
            return True
    return False


def _sorted_names(path: str) -> list[str]:
    # readDirNames + sort.Strings: byte-wise order.
    names = os.listdir(path)
    names.sort(key=lambda n: os.fsencode(n))
    return names


def dir_media(path: str) -> list[str]:
    """Return media files below ``path`` (Go ``process.Dir``)."""
    with os.scandir(path) as it:  # raises FileNotFoundError / NotADirectoryError
        top_dirs = [e.name for e in it if e.is_dir(follow_symlinks=False)]
    allowed: tuple[str, ...] = ALLOWED_DIRS
    if len(top_dirs) == 1:
        allowed = allowed + (top_dirs[0],)

    files: list[str] = []

    def walk(p: str, is_root: bool) -> None:
        # p is a directory that has been admitted.
        try:
            names = _sorted_names(p)
        except OSError:
            if is_root:
                raise
            return  # reference: allowed dir with readdir error → walkFn nil → skipped
        for name in names:
            full = go_join(p, name)
            st = os.lstat(full)  # error propagates (B11 fix)
            if stat.S_ISDIR(st.st_mode):
                if _dir_allowed(go_base(full), allowed):
                    walk(full, False)
                continue
            if go_ext(full) in MEDIA_EXTS:
                files.append(full)

    walk(path, True)
    return files


def predict_media(path: str, files: list[str]) -> set[str] | None:
    """What :func:`dir_media` will return for ``files`` (absolute paths below
    ``path``) once they exist — evaluated on the path strings alone, so a
    torrent's media files can be uploaded as each completes.

    Only directories change the rules (the sole-top-level-directory
    allow-list entry), so the prediction is exact when every directory that
    exists under ``path`` now is one the torrent itself creates; any other
    top-level directory returns ``None`` (the caller must wait for the real
    walk).  Plain files that are not in ``files`` never change the answer for
    the files that are."""
    root = go_join(path)
    rels: list[list[str]] = []
    for f in files:
        p = go_join(f)
        if not p.startswith(root.rstrip("/") + "/"):
            return None
        rels.append(p[len(root.rstrip("/")) + 1:].split("/"))
    tops = {r[0] for r in rels if len(r) > 1}
    try:
        with os.scandir(path) as it:
            present = {e.name for e in it if e.is_dir(follow_symlinks=False)}
    except FileNotFoundError:
        present = set()
    if not present <= tops:
        return None
    allowed: tuple[str, ...] = ALLOWED_DIRS
    if len(tops) == 1:
        allowed = allowed + (next(iter(tops)),)
    out: set[str] = set()
    for r in rels:
        full = go_join(root, *r)
        if go_ext(full) in MEDIA_EXTS and all(_dir_allowed(c, allowed) for c in r[:-1]):
            out.add(full)
    return out


# Reference-compatible alias: ``process.Dir``.
Dir = dir_media
