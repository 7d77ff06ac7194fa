#!/usr/bin/env python3
"""Tiny undefined-name check (no pyflakes in the image): flags names loaded inside a function that
are neither assigned/imported there nor defined at module level nor builtins."""
import ast
import builtins
import sys


def check(path):
    tree = ast.parse(open(path).read())
    glob = set()
    for n in ast.walk(tree):
        if isinstance(n, (ast.FunctionDef, ast.ClassDef, ast.AsyncFunctionDef)):
            glob.add(n.name)
        if isinstance(n, (ast.Import, ast.ImportFrom)) and n in tree.body:
            for a in n.names:
                glob.add((a.asname or a.name).split(".")[0])
        if isinstance(n, ast.Assign) and n in tree.body:
            for t in n.targets:
                for m in ast.walk(t):
                    if isinstance(m, ast.Name):
                        glob.add(m.id)
        if isinstance(n, (ast.AnnAssign,)) and n in tree.body and isinstance(n.target, ast.Name):
            glob.add(n.target.id)
    bad = []
    for fn in ast.walk(tree):
        if not isinstance(fn, (ast.FunctionDef, ast.AsyncFunctionDef)):
            continue
        assigned = set()
        for n in ast.walk(fn):
            if isinstance(n, ast.arg):
                assigned.add(n.arg)
            if isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
                assigned.add(n.id)
            if isinstance(n, (ast.Import, ast.ImportFrom)):
                for a in n.names:
                    assigned.add((a.asname or a.name).split(".")[0])
            if isinstance(n, ast.ExceptHandler) and n.name:
                assigned.add(n.name)
            if isinstance(n, (ast.Global, ast.Nonlocal)):
                assigned.update(n.names)
        # names assigned in enclosing functions
        for outer in ast.walk(tree):
            if isinstance(outer, (ast.FunctionDef, ast.AsyncFunctionDef)) and outer is not fn and fn in ast.walk(outer):
                for n in ast.walk(outer):
                    if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Store):
                        assigned.add(n.id)
                    if isinstance(n, ast.arg):
                        assigned.add(n.arg)
                    if isinstance(n, (ast.Import, ast.ImportFrom)):
                        for a in n.names:
                            assigned.add((a.asname or a.name).split(".")[0])
        for n in ast.walk(fn):
            if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load):
                if n.id not in assigned and n.id not in glob and not hasattr(builtins, n.id) and n.id != "__file__":
                    bad.append(f"{path}:{n.lineno}: undefined name {n.id!r} in {fn.name}")
    return bad


if __name__ == "__main__":
    out = []
    for p in sys.argv[1:]:
        out += check(p)
    print("\n".join(sorted(set(out))))
    sys.exit(1 if out else 0)
