"""Tabulate bench runs against where they were placed.

For each ``bench.py`` log (or ``runs.jsonl`` row) prints the job rate, the
L3 domain the worker was pinned to and how busy that domain and the fakes'
domain were when the run was placed (``placement.ccd_busy_at_launch``, sampled
over 0.2 s before pinning, other tenants of the host included).  Used to
check whether slow runs on a shared host were the ones placed on domains
another tenant was using.

    python tools/placement_table.py profiles/r06_final4/runs.jsonl profiles/r06_final4/*/runs.jsonl
"""

from __future__ import annotations

import json
import os
import sys


def _records(path: str):
    with open(path) as f:
        lines = [ln for ln in f if ln.strip()]
    if path.endswith(".jsonl"):
        for ln in lines:
            r = json.loads(ln)
            yield f"{os.path.basename(os.path.dirname(os.path.abspath(path)))}/{r.get('log', '')}", r
        return
    recs = [ln for ln in lines if ln.startswith('{"metric"')]
    if recs:
        yield os.path.basename(path)[:-4], json.loads(recs[-1])


def _placement(r: dict) -> dict:
    for v in r.values():
        if isinstance(v, dict) and "chosen_ccds" in v:
            return v
    return {}


def main(paths: list[str]) -> int:
    rows = []
    for p in paths:
        for name, r in _records(p):
            pl = _placement(r)
            busy = pl.get("ccd_busy_at_launch", {})
            ccds = pl.get("chosen_ccds") or []
            fake = pl.get("fake_ccd")
            mine = max((busy.get(str(c), 0.0) for c in ccds), default=None)
            idle = sum(1 for b in busy.values() if b <= 0.01)
            rows.append((name, r.get("value"), ccds, mine, fake, busy.get(str(fake)) if fake is not None else None,
                         idle, len(busy)))
    print("| run | jobs/s | worker L3 (first CPU) | its busy | fakes L3 | its busy | domains <= 1 % busy |")
    print("|---|---|---|---|---|---|---|")
    for name, v, ccds, mine, fake, fb, idle, n in rows:
        print(f"| {name} | {v:.1f} | {','.join(map(str, ccds))} | {mine if mine is not None else '-'} | "
              f"{fake if fake is not None else '-'} | {fb if fb is not None else '-'} | {idle} of {n} |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
