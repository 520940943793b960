"""Crude undefined-global check for the csu modules (no pyflakes in the image): names loaded anywhere
that are never bound anywhere in the module (assignment, argument, import, def, comprehension)."""
import ast
import builtins
import sys

for path in sys.argv[1:]:
    tree = ast.parse(open(path).read())
    bound, used = set(dir(builtins)), {}
    for n in ast.walk(tree):
        if isinstance(n, ast.Name):
            if isinstance(n.ctx, ast.Load):
                used.setdefault(n.id, n.lineno)
            else:
                bound.add(n.id)
        elif isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            bound.add(n.name)
        elif isinstance(n, ast.arg):
            bound.add(n.arg)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            for a in n.names:
                bound.add((a.asname or a.name).split(".")[0])
        elif isinstance(n, ast.ExceptHandler) and n.name:
            bound.add(n.name)
    for k, ln in sorted(used.items(), key=lambda kv: kv[1]):
        if k not in bound:
            print(f"{path}:{ln}: undefined name {k}")
