"""Collapse a profiles/ directory's bench logs into one ``runs.jsonl``.

Each ``bench.py`` log ends with its JSON record (the driver contract line,
with ``config``, ``diag``, ``noise`` and CPU per job).  That record is the
evidence a summary cites; the progress lines above it are not.  This
writes one JSON line per log, ``{"log": <log stem>, **record}``, removes
those logs, and points the directory's SUMMARY.md at ``runs.jsonl``.
Logs whose last line is not a bench record (pytest, smoke, soak) stay.

    python tools/collapse_logs.py profiles/r06_noise profiles/r06_final ...
"""

from __future__ import annotations

import glob
import json
import os
import re
import sys


def _is_bench(path: str) -> bool:
    with open(path) as f:
        first = f.readline()
    return not first.strip() or '"metric"' in first


def collapse(d: str) -> int:
    rows = []
    done = []
    for path in sorted(glob.glob(os.path.join(d, "*.log"))):
        try:
            with open(path) as f:
                lines = [ln for ln in f.read().splitlines() if ln.strip()]
            rec = json.loads(lines[-1]) if lines else None
        except (OSError, ValueError):
            continue
        if not isinstance(rec, dict) or "metric" not in rec:
            continue
        if sum(ln.startswith('{"metric"') for ln in lines) > 1:
            continue                                # several records (e.g. bench_resume): keep the log
        rows.append({"log": os.path.basename(path)[:-4], **rec})
        done.append(path)
    if not rows:
        return 0
    out = os.path.join(d, "runs.jsonl" if not os.path.exists(os.path.join(d, "runs.jsonl"))
                       or _is_bench(os.path.join(d, "runs.jsonl")) else "bench_runs.jsonl")
    old = []
    if os.path.exists(out):
        with open(out) as f:
            old = [json.loads(ln) for ln in f if ln.strip()]
    with open(out, "w") as f:
        for r in old + rows:
            f.write(json.dumps(r) + "\n")
    for p in done:
        os.remove(p)
    summ = os.path.join(d, "SUMMARY.md")
    if os.path.exists(summ):
        with open(summ) as f:
            text = f.read()
        names = {os.path.basename(p)[:-4] for p in done}
        text = re.sub(r"`([\w.-]+)\.log`", lambda m: f"`{m.group(1)}` in `runs.jsonl`" if m.group(1) in names
                      else m.group(0), text)
        if "runs.jsonl" not in text:
            text += ("\nEach run's bench record (its JSON line, with config, diag and CPU per job) is in "
                     "`runs.jsonl`, keyed by the log name (`log`).\n")
        with open(summ, "w") as f:
            f.write(text)
    return len(rows)


def main() -> int:
    for d in sys.argv[1:]:
        print(d, collapse(d))
    return 0


if __name__ == "__main__":
    sys.exit(main())
