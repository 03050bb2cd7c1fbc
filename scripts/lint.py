#!/usr/bin/env python3
"""Dependency-free lint for the repository's Python and C++/HIP sources (the image has no ruff /
flake8; CI runs this same script).  Checks:

* every .py compiles;
* unused imports (module-level and function-level ``import x`` / ``from y import x`` whose name is
  never referenced; ``__init__`` re-exports, ``# noqa`` lines and ``__future__`` are exempt);
* no tabs, no trailing whitespace, lines <= 120 chars (Python) / 120 (C++/HIP), newline at EOF;
* no ``print(`` debugging left in the library package (arbius_amd/, except the CLI).

    python scripts/lint.py [paths...]     # exit 1 on any finding
"""
from __future__ import annotations

import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY_DIRS = ("arbius_amd", "tests", "scripts")
PY_FILES = ("bench.py", "__graft_entry__.py")
CPP_EXT = (".hip", ".h", ".inc", ".cpp")
MAXLEN = 120


def _names_used(tree) -> set:
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            base = node
            while isinstance(base, ast.Attribute):
                base = base.value
            if isinstance(base, ast.Name):
                used.add(base.id)
    # names referenced in __all__ strings and string annotations
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str) and node.value.isidentifier():
            used.add(node.value)
    return used


def lint_py(path: str, rel: str) -> list:
    out = []
    src = open(path, encoding="utf-8").read()
    try:
        tree = ast.parse(src, filename=rel)
    except SyntaxError as e:
        return [f"{rel}:{e.lineno}: syntax error: {e.msg}"]
    lines = src.split("\n")
    if src and not src.endswith("\n"):
        out.append(f"{rel}: no newline at end of file")
    for i, line in enumerate(lines, 1):
        if "\t" in line:
            out.append(f"{rel}:{i}: tab character")
        if line.rstrip() != line:
            out.append(f"{rel}:{i}: trailing whitespace")
        if len(line) > MAXLEN and "noqa" not in line and "http" not in line:
            out.append(f"{rel}:{i}: line longer than {MAXLEN} ({len(line)})")
    if os.path.basename(path) == "__init__.py":
        return out                      # package re-exports
    used = _names_used(tree)
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            line = lines[node.lineno - 1]
            if "noqa" in line:
                continue
            for a in node.names:
                name = (a.asname or a.name).split(".")[0]
                if name != "*" and name not in used:
                    out.append(f"{rel}:{node.lineno}: unused import {name}")
    if rel.startswith("arbius_amd/") and rel not in ("arbius_amd/cli.py", "arbius_amd/__main__.py") \
            and not rel.endswith(("build.py",)):
        for node in ast.walk(tree):
            if isinstance(node, ast.Call) and isinstance(node.func, ast.Name) and node.func.id == "print":
                if "noqa" not in lines[node.lineno - 1]:
                    out.append(f"{rel}:{node.lineno}: print() in library code (use logging)")
    return out


def lint_cpp(path: str, rel: str) -> list:
    out = []
    src = open(path, encoding="utf-8").read()
    if src and not src.endswith("\n"):
        out.append(f"{rel}: no newline at end of file")
    for i, line in enumerate(src.split("\n"), 1):
        if "\t" in line:
            out.append(f"{rel}:{i}: tab character")
        if line.rstrip() != line:
            out.append(f"{rel}:{i}: trailing whitespace")
        if len(line) > MAXLEN:
            out.append(f"{rel}:{i}: line longer than {MAXLEN} ({len(line)})")
    return out


def files(paths):
    if paths:
        for p in paths:
            yield os.path.abspath(p)
        return
    for d in PY_DIRS:
        for dp, dn, fn in os.walk(os.path.join(ROOT, d)):
            dn[:] = [x for x in dn if not x.startswith((".", "__pycache__", "build_obj"))]
            for f in sorted(fn):
                if f.endswith(".py") or f.endswith(CPP_EXT):
                    yield os.path.join(dp, f)
    for f in PY_FILES:
        yield os.path.join(ROOT, f)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    findings = []
    n = 0
    for path in files(argv):
        rel = os.path.relpath(path, ROOT)
        n += 1
        findings += lint_py(path, rel) if path.endswith(".py") else lint_cpp(path, rel)
    for f in findings:
        print(f)
    print(f"lint: {n} files, {len(findings)} findings")
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main())
