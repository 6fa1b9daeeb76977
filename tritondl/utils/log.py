"""logrus-compatible structured logging (reference C12,
``cmd/downloader/downloader.go:45-52``).

* text (default): ``time="2006-01-02T15:04:05Z07:00" level=info msg="..." k=v``
* ``LOG_FORMAT=json``: ``{"level":"info","msg":"...","time":"...",k:v}``
* ``LOG_LEVEL=debug``: caller reporting (``func=``/``file=``) as logrus
  ``SetReportCaller(true)``, and — unlike the reference (B10) — the level is
  lowered to debug as well.

Thread-safe: one lock around the final write, so worker threads (native
hashing callbacks, torch.distributed ranks) never interleave lines.
"""

from __future__ import annotations

import json
import re
import sys
import threading
import time
from typing import Any, TextIO

# scheme://user:password@ in any line (a source URL with credentials, the AMQP
# URL) is written as scheme://user:xxxxx@, as Go's url.URL.Redacted()
_CREDS = re.compile(r"([A-Za-z][A-Za-z0-9+.-]*://[^/\s:@\"]*):[^@\s/\"]+@")

LEVELS = {"trace": 6, "debug": 5, "info": 4, "warning": 3, "error": 2, "fatal": 1, "panic": 0}


_ts_cache: tuple[int, str] = (-1, "")


def _fmt_ts(t: float) -> str:
    global _ts_cache
    sec = int(t)                        # the string changes once a second: build it once
    if _ts_cache[0] == sec:
        return _ts_cache[1]
    lt = time.localtime(t)
    off = lt.tm_gmtoff or 0
    if off == 0:
        z = "Z"
    else:
        s = "+" if off > 0 else "-"
        off = abs(off)
        z = f"{s}{off // 3600:02d}:{(off % 3600) // 60:02d}"
    out = time.strftime("%Y-%m-%dT%H:%M:%S", lt) + z
    _ts_cache = (sec, out)
    return out


def _needs_quote(s: str) -> bool:
    if s == "":
        return True
    for ch in s:
        if not (ch.isalnum() or ch in "-._/@^+"):
            return True
    return False


def _text_value(v: Any) -> str:
    if isinstance(v, BaseException):
        v = str(v)
    if not isinstance(v, str):
        if isinstance(v, (list, tuple)):
            v = "[" + " ".join(str(x) for x in v) + "]"
        else:
            v = str(v)
    return json.dumps(v) if _needs_quote(v) else v


def _json_value(v: Any) -> Any:
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    if isinstance(v, (list, tuple)):
        return [_json_value(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _json_value(x) for k, x in v.items()}
    if hasattr(v, "to_dict"):
        return v.to_dict()
    return str(v)


class Logger:
    def __init__(self, stream: TextIO | None = None) -> None:
        self.stream = stream
        self.level = LEVELS["info"]
        self.json = False
        self.report_caller = False
        self._lock = threading.Lock()

    def configure(self, log_level: str = "", log_format: str = "") -> None:
        if log_level.lower() == "debug":
            self.report_caller = True
            self.level = LEVELS["debug"]
        elif log_level.lower() in LEVELS:
            self.level = LEVELS[log_level.lower()]
        self.json = log_format.lower() == "json"

    # entry constructors -------------------------------------------------
    def with_field(self, key: str, value: Any) -> "Entry":
        return Entry(self, {key: value})

    def with_fields(self, fields: dict | None = None, **kw: Any) -> "Entry":
        d = dict(fields or {})
        d.update(kw)
        return Entry(self, d)

    def enabled(self, level: str) -> bool:
        """Would a record at ``level`` be emitted?  (Guards costly field building.)"""
        return LEVELS[level] <= self.level

    # direct logging ----------------------------------------------------
    # debug/info are called on every job: a disabled level returns before
    # building an entry or formatting the message
    def debug(self, msg: str, *a: Any) -> None:
        if LEVELS["debug"] <= self.level:
            Entry(self, {})._log("debug", msg, a, 3)

    def info(self, msg: str, *a: Any) -> None:
        if LEVELS["info"] <= self.level:
            Entry(self, {})._log("info", msg, a, 3)

    def warn(self, msg: str, *a: Any) -> None:
        Entry(self, {})._log("warning", msg, a, 3)

    warning = warn

    def error(self, msg: str, *a: Any) -> None:
        Entry(self, {})._log("error", msg, a, 3)

    def fatal(self, msg: str, *a: Any) -> None:
        Entry(self, {})._log("fatal", msg, a, 3)
        raise SystemExit(1)

    def _emit(self, level: str, msg: str, fields: dict, depth: int) -> None:
        if LEVELS[level] > self.level:
            return
        now = time.time()
        rec: dict[str, Any] = {}
        if self.report_caller:
            f = sys._getframe(depth)
            rec["func"] = f"{f.f_globals.get('__name__', '?')}.{f.f_code.co_name}"
            rec["file"] = f"{f.f_code.co_filename}:{f.f_lineno}"
        if self.json:
            out: dict[str, Any] = {k: _json_value(v) for k, v in fields.items()}
            out.update({"level": level, "msg": msg, "time": _fmt_ts(now)})
            out.update(rec)
            line = json.dumps(out, sort_keys=True)
        else:
            parts = [f'time="{_fmt_ts(now)}"', f"level={level}", f"msg={_text_value(msg)}"]
            parts += [f"{k}={_text_value(v)}" for k, v in sorted(fields.items())]
            parts += [f"{k}={_text_value(v)}" for k, v in rec.items()]
            line = " ".join(parts)
        if "@" in line:
            line = _CREDS.sub(r"\1:xxxxx@", line)
        stream = self.stream or sys.stderr
        with self._lock:
            stream.write(line + "\n")
            try:
                stream.flush()
            except Exception:
                pass


class Entry:
    __slots__ = ("logger", "fields")

    def __init__(self, logger: Logger, fields: dict) -> None:
        self.logger = logger
        self.fields = fields

    def with_field(self, key: str, value: Any) -> "Entry":
        d = dict(self.fields)
        d[key] = value
        return Entry(self.logger, d)

    def with_fields(self, fields: dict | None = None, **kw: Any) -> "Entry":
        d = dict(self.fields)
        d.update(fields or {})
        d.update(kw)
        return Entry(self.logger, d)

    def _log(self, level: str, msg: str, args: tuple, depth: int) -> None:
        if LEVELS[level] > self.logger.level:
            return
        if args:
            msg = msg % args
        self.logger._emit(level, msg, self.fields, depth + 1)

    def debug(self, msg: str, *a: Any) -> None:
        self._log("debug", msg, a, 2)

    def info(self, msg: str, *a: Any) -> None:
        self._log("info", msg, a, 2)

    def warn(self, msg: str, *a: Any) -> None:
        self._log("warning", msg, a, 2)

    warning = warn

    def error(self, msg: str, *a: Any) -> None:
        self._log("error", msg, a, 2)


log = Logger()
