#!/usr/bin/env python3
"""Minimal static checks with the standard library only (no linters are
installed in the build image): every file compiles, no module imports a
name it never uses, no function reads a global the module never binds, and
every ``profiles/`` path the docs and code cite exists
(``tools/prune_profiles.py --check``).  ``__init__.py`` re-exports and names listed in
``__all__`` count as used; ``# noqa`` on the import line skips it.

    python tools/lint.py [paths...]        # exit 1 and one line per finding
"""

from __future__ import annotations

import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = ["tritondl", "tritondl_testkit", "tests", "tools", "bench.py", "__graft_entry__.py"]


def _files(paths: list[str]):
    for p in paths:
        p = os.path.join(ROOT, p) if not os.path.isabs(p) else p
        if os.path.isfile(p) and p.endswith(".py"):
            yield p
            continue
        for root, dirs, files in os.walk(p):
            dirs[:] = [d for d in dirs if d not in ("__pycache__", ".ab", "build")]
            for f in files:
                if f.endswith(".py"):
                    yield os.path.join(root, f)


def unused_imports(path: str, src: str) -> list[str]:
    tree = ast.parse(src, path)
    if os.path.basename(path) == "__init__.py":
        return []
    lines = src.splitlines()
    imported: dict[str, int] = {}
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            if "noqa" in lines[node.lineno - 1]:
                continue
            for a in node.names:
                if a.name == "*":
                    continue
                name = a.asname or a.name.split(".")[0]
                imported.setdefault(name, node.lineno)
    used: set[str] = set()
    strings: list[str] = []          # string annotations ("Foo | None") and __all__ entries
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            base = node
            while isinstance(base, ast.Attribute):
                base = base.value
            if isinstance(base, ast.Name):
                used.add(base.id)
        ann = []
        if isinstance(node, ast.arg) and node.annotation is not None:
            ann.append(node.annotation)
        elif isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)) and node.returns is not None:
            ann.append(node.returns)
        elif isinstance(node, ast.AnnAssign):
            ann.append(node.annotation)
        elif isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            ann.append(node.value)
        for a in ann:
            strings += [c.value for c in ast.walk(a) if isinstance(c, ast.Constant) and isinstance(c.value, str)]
    for text in strings:
        for tok in text.replace("[", " ").replace("]", " ").replace("|", " ").replace(",", " ").split():
            used.add(tok.split(".")[0].strip("'\""))
    return [f"{path}:{ln}: '{name}' imported but unused" for name, ln in sorted(imported.items(), key=lambda x: x[1])
            if name not in used]


def undefined_globals(path: str, src: str) -> list[str]:
    """Names a function or class body reads as globals that the module never
    binds and that are not builtins (a missing import, a typo): what a
    NameError at run time would be.  From the compiler's own symbol tables."""
    import builtins
    import symtable
    top = symtable.symtable(src, path, "exec")
    bound = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()
             or s.is_namespace() or s.is_parameter()}
    if any(s.get_name() == "*" for s in top.get_symbols()) or "__getattr__" in bound:
        return []
    known = bound | set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__spec__", "__builtins__",
                                          "__path__", "__package__", "__loader__", "__class__"}
    out = []

    def walk(t) -> None:
        for c in t.get_children():
            for sym in c.get_symbols():
                if sym.is_referenced() and (sym.is_global() or sym.is_declared_global()) \
                        and sym.get_name() not in known:
                    out.append(f"{path}: '{sym.get_name()}' is used in {c.get_name()}() but never defined")
            walk(c)
    walk(top)
    return sorted(set(out))


def main(argv: list[str]) -> int:
    paths = argv or DEFAULT
    problems: list[str] = []
    for f in _files(paths):
        with open(f, encoding="utf-8") as fh:
            src = fh.read()
        try:
            compile(src, f, "exec")
        except SyntaxError as e:
            problems.append(f"{f}:{e.lineno}: {e.msg}")
            continue
        problems += unused_imports(f, src)
        problems += undefined_globals(f, src)
    if not argv:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from prune_profiles import check_citations
        problems += [f"cited but missing: {m}" for m in check_citations()]
    for p in problems:
        print(os.path.relpath(p, ROOT) if p.startswith(ROOT) else p)
    return 1 if problems else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
