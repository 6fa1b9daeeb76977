"""Small helpers reproducing Go stdlib semantics the wire contract depends on.

* ``go_ext``    – ``path/filepath.Ext`` (Python's ``splitext`` differs on
                  dot-files: Go's ``Ext(".mkv") == ".mkv"``).
* ``go_clean`` / ``go_join`` – ``path.Clean`` / ``filepath.Join`` (lexical).
* ``go_time_string`` – ``time.Now().String()`` as used for
  ``Convert.CreatedAt`` (reference ``cmd/downloader/downloader.go:137``).
"""

from __future__ import annotations

import time


def go_ext(path: str) -> str:
    """filepath.Ext: suffix starting at the final dot of the final element."""
    i = len(path) - 1
    while i >= 0 and path[i] != "/":
        if path[i] == ".":
            return path[i:]
        i -= 1
    return ""


def go_clean(path: str) -> str:
    """path.Clean (lexical processing, Go semantics)."""
    if path == "":
        return "."
    rooted = path.startswith("/")
    out: list[str] = []
    for part in path.split("/"):
        if part in ("", "."):
            continue
        if part == "..":
            if out and out[-1] != "..":
                out.pop()
            elif not rooted:
                out.append("..")
            continue
        out.append(part)
    res = "/".join(out)
    if rooted:
        return "/" + res
    return res or "."


def go_join(*elems: str) -> str:
    """filepath.Join: join non-empty elements with '/', then Clean."""
    parts = [e for e in elems if e != ""]
    if not parts:
        return ""
    return go_clean("/".join(parts))


def go_base(path: str) -> str:
    """filepath.Base."""
    if path == "":
        return "."
    path = path.rstrip("/")
    if path == "":
        return "/"
    i = path.rfind("/")
    return path[i + 1:] if i >= 0 else path


_T0_NS = time.monotonic_ns()


def go_time_string(now_ns: int | None = None, mono_ns: int | None = None) -> str:
    """Format like Go's ``time.Time.String()`` for ``time.Now()``.

    ``2006-01-02 15:04:05.999999999 -0700 MST m=+0.000000001``: fractional
    seconds with trailing zeros trimmed, numeric zone, zone abbreviation and
    the monotonic-clock reading relative to process start.
    """
    if now_ns is None:
        now_ns = time.time_ns()
    if mono_ns is None:
        mono_ns = time.monotonic_ns() - _T0_NS
    secs, frac = divmod(now_ns, 1_000_000_000)
    lt = time.localtime(secs)
    base = time.strftime("%Y-%m-%d %H:%M:%S", lt)
    if frac:
        base += ("." + f"{frac:09d}").rstrip("0")
    off = lt.tm_gmtoff or 0
    sign = "+" if off >= 0 else "-"
    off = abs(off)
    zone = f"{sign}{off // 3600:02d}{(off % 3600) // 60:02d}"
    abbr = lt.tm_zone or "UTC"
    ms, mfrac = divmod(mono_ns, 1_000_000_000)
    return f"{base} {zone} {abbr} m=+{ms}.{mfrac:09d}"


_DURAFMT_UNITS = [("year", 365 * 24 * 3600 * 10**6), ("week", 7 * 24 * 3600 * 10**6), ("day", 24 * 3600 * 10**6),
                  ("hour", 3600 * 10**6), ("minute", 60 * 10**6), ("second", 10**6), ("millisecond", 1000),
                  ("microsecond", 1)]


def durafmt(seconds: float) -> str:
    """``durafmt.Parse(d).String()`` (hako/durafmt, used for the reference's
    "retrying message in %s" log line, ``internal/rabbitmq/client.go:208``):
    every non-zero unit from years down to microseconds, singular/plural,
    space separated; ``0 seconds`` for zero."""
    us = int(round(abs(seconds) * 1_000_000))
    parts = []
    for name, n in _DURAFMT_UNITS:
        q, us = divmod(us, n)
        if q:
            parts.append(f"{q} {name}" + ("" if q == 1 else "s"))
    if not parts:
        return "0 seconds"
    return ("-" if seconds < 0 else "") + " ".join(parts)
