#!/usr/bin/env python3
"""Prune ``profiles/`` to the evidence the docs and code cite.

Every directory of ``profiles/`` that README.md, docs/*.md, VERDICT.md or
the code cite keeps its ``SUMMARY.md`` (a digest of the numbers in its raw
logs is written where it had none) and every file cited by name; the raw
logs go.  Directories nothing cites are removed.  ``profiles/ARCHIVE.md``
lists what was removed and the commit that still holds it (``git show
<commit>:<path>``).  :func:`check_citations` (run by ``tools/lint.py``)
fails when a cited ``profiles/`` path is missing.

    python tools/prune_profiles.py            # prune (then commit)
    python tools/prune_profiles.py --check    # citation check only
"""

from __future__ import annotations

import json
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
_CITE = re.compile(r"profiles/[A-Za-z0-9_./*-]+")
# where citations count: the docs a reader follows and the code's own comments
SOURCES = ["README.md", "VERDICT.md", "SURVEY.md", "BASELINE.md", "docs", "tritondl", "tritondl_testkit", "tools",
           "tests", "csrc", "bench.py", "__graft_entry__.py", "Makefile", "hack"]
KEEP_ALWAYS = {"README.md", "ARCHIVE.md"}


def _files(rel: str):
    p = os.path.join(ROOT, rel)
    if os.path.isfile(p):
        yield p
        return
    for root, dirs, files in os.walk(p):
        dirs[:] = [d for d in dirs if d not in ("__pycache__", ".git")]
        for f in files:
            if f.endswith((".py", ".md", ".h", ".cpp", ".hip", ".sh", ".txt", ".toml", ".yml")) or f == "Makefile":
                yield os.path.join(root, f)


def citations() -> set[str]:
    out = set()
    for rel in SOURCES:
        for path in _files(rel):
            if os.path.abspath(path).startswith(os.path.abspath(PROF)):
                continue
            try:
                text = open(path, encoding="utf-8", errors="replace").read()
            except OSError:
                continue
            for m in _CITE.finditer(text):
                c = m.group(0).rstrip(".,:;)`'\"")
                out.add(c)
    return out


def _expand(c: str) -> list[str]:
    """A citation's concrete paths: ``r04_fresh1..5/`` names five dirs;
    a bare prefix (``profiles/r03_``) names none."""
    m = re.match(r"(profiles/[A-Za-z0-9_]+?)(\d+)\.\.(\d+)(/.*)?$", c)
    if m:
        base, a, b, rest = m.group(1), int(m.group(2)), int(m.group(3)), m.group(4) or "/"
        rest = "/" if rest.endswith("_") or "_" in rest.rsplit("/", 1)[-1] and not rest.endswith(".md") else rest
        return [f"{base}{i}{rest}" for i in range(a, b + 1)]
    tail = c.split("/", 1)[1] if "/" in c else ""
    if not tail or tail.endswith("_") or re.fullmatch(r"r\d+", tail):
        return []
    return [c]


def _exists(p: str) -> bool:
    import glob
    full = os.path.join(ROOT, p.rstrip("/"))
    return bool(glob.glob(full)) if "*" in p else os.path.exists(full)


def check_citations() -> list[str]:
    """Cited profiles paths that do not exist (``*`` globs must match)."""
    missing = []
    for c in sorted(citations()):
        for p in _expand(c):
            if not _exists(p):
                missing.append(p)
    return missing


def _digest(d: str) -> str:
    """Numbers from a run dir's raw logs: each bench JSON line's headline, and
    the last line of every other log."""
    lines = []
    for root, _dirs, files in os.walk(d):
        for f in sorted(files):
            p = os.path.join(root, f)
            rel = os.path.relpath(p, d)
            try:
                text = open(p, encoding="utf-8", errors="replace").read()
            except OSError:
                continue
            got = False
            for ln in text.splitlines():
                if ln.startswith("{") and '"value"' in ln:
                    try:
                        j = json.loads(ln)
                    except ValueError:
                        continue
                    cfg = j.get("config") or {}
                    lines.append(f"| `{rel}` | {j.get('metric')} {j.get('value')} {j.get('unit', '')} | steps "
                                 f"{j.get('steps')}, concurrency {cfg.get('concurrency_per_worker')}, "
                                 f"{cfg.get('transport', '')} {cfg.get('file_bytes', '')} B |")
                    got = True
            if not got:
                last = [ln for ln in text.splitlines() if ln.strip()][-1:] or [""]
                lines.append(f"| `{rel}` | {last[0][:160].replace('|', '/')} | |")
            if len(lines) >= 80:
                lines.append("| ... | (more files in the archive) | |")
                return "\n".join(lines)
    return "\n".join(lines)


def prune(commit: str) -> tuple[int, list[str]]:
    import glob
    cited = set()
    for c in citations():
        for p in _expand(c):
            if "*" in p:
                cited.update(os.path.relpath(g, ROOT) for g in glob.glob(os.path.join(ROOT, p)))
            else:
                cited.add(p.rstrip("/"))
    removed: list[str] = []
    for name in sorted(os.listdir(PROF)):
        d = os.path.join(PROF, name)
        rel = f"profiles/{name}"
        if not os.path.isdir(d):
            continue
        keep_files = {p for p in cited if p == rel or p.startswith(rel + "/")}
        if not keep_files:
            first = ""
            s = os.path.join(d, "SUMMARY.md")
            if os.path.exists(s):
                first = next((ln.strip("# ").strip() for ln in open(s) if ln.strip()), "")
            removed.append(f"| `{rel}/` | {first[:120]} |")
            shutil.rmtree(d)
            continue
        keep = {os.path.join(ROOT, p) for p in keep_files if p != rel}
        # cited sub-directories keep their own summary, like a top-level one
        summaries = [d] + [os.path.join(ROOT, p) for p in keep_files if os.path.isdir(os.path.join(ROOT, p))]
        for sd in summaries:
            s = os.path.join(sd, "SUMMARY.md")
            if not os.path.exists(s):
                body = _digest(sd)
                with open(s, "w") as f:
                    f.write(f"# {os.path.relpath(sd, ROOT)} (digest)\n\nGenerated when the raw logs were pruned; "
                            f"they are in commit `{commit}` (`git show {commit}:{os.path.relpath(sd, ROOT)}/<file>`)."
                            f"\n\n| file | result | |\n|---|---|---|\n{body}\n")
            keep.add(s)
        for root, _dirs, files in os.walk(d, topdown=False):
            for f in files:
                p = os.path.join(root, f)
                if p not in keep and not any(p.startswith(k.rstrip("/") + "/") and os.path.isdir(k) and
                                            os.path.basename(p) == "SUMMARY.md" for k in keep):
                    os.remove(p)
            if not os.listdir(root):
                os.rmdir(root)
    return len(removed), removed


def main() -> int:
    if "--check" in sys.argv:
        miss = check_citations()
        for m in miss:
            print(f"missing cited path: {m}")
        return 1 if miss else 0
    commit = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], cwd=ROOT, capture_output=True,
                            text=True).stdout.strip()
    n, removed = prune(commit)
    arch = os.path.join(PROF, "ARCHIVE.md")
    old = open(arch).read() if os.path.exists(arch) else (
        "# Archived profiles\n\nRun directories nothing in README.md, docs/ or the code cites any more, and the raw "
        "logs of the cited ones, were removed from the tree.  Each is still in git history: "
        "`git show <commit>:profiles/<dir>/<file>` (`git ls-tree -r --name-only <commit> profiles/<dir>`).\n")
    with open(arch, "w") as f:
        f.write(old.rstrip("\n") + f"\n\n## Removed at `{commit}`\n\n| directory | summary |\n|---|---|\n"
                + "\n".join(removed) + "\n")
    print(f"removed {n} directories; raw logs of the cited ones pruned (archive: {commit})")
    miss = check_citations()
    for m in miss:
        print(f"missing cited path: {m}")
    return 1 if miss else 0


if __name__ == "__main__":
    sys.exit(main())
