"""Undefined-name check for the Python sources (no pyflakes in this image).

    python tools/lint_names.py [files...]     (default: pbn_rl_amd/*.py, bench.py, tools/*.py)

Reports every name a function body loads that is neither bound in an enclosing function
scope, nor a module-level binding, nor a builtin.  Catches the edit slips (a renamed local)
that otherwise only surface on the GPU box.  Exit status 1 if anything is reported.
"""
import ast
import builtins
import glob
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def bound_names(node):
    """Names bound directly in a scope node (not in nested function/class scopes)."""
    out = set()
    if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
        a = node.args
        for arg in a.posonlyargs + a.args + a.kwonlyargs:
            out.add(arg.arg)
        if a.vararg:
            out.add(a.vararg.arg)
        if a.kwarg:
            out.add(a.kwarg.arg)
    body = node.body if isinstance(node.body, list) else [node.body]
    stack = list(body)
    while stack:
        n = stack.pop()
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out.add(n.name)
            stack.extend(n.decorator_list)
            continue
        if isinstance(n, ast.Lambda):
            continue
        if isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            out.add(n.id)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            for al in n.names:
                out.add((al.asname or al.name).split(".")[0])
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            out.update(n.names)
        elif isinstance(n, ast.ExceptHandler) and n.name:
            out.add(n.name)
        elif isinstance(n, ast.NamedExpr):
            out.add(n.target.id)
        elif isinstance(n, ast.arg):
            out.add(n.arg)
        stack.extend(ast.iter_child_nodes(n))
    return out


def check(path):
    with open(path) as f:
        tree = ast.parse(f.read(), path)
    problems = []
    module_names = bound_names(tree) | set(dir(builtins)) | {"__file__", "__name__", "__doc__"}

    def visit(node, scopes):
        for child in ast.iter_child_nodes(node):
            if isinstance(child, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
                visit(child, scopes + [bound_names(child)])
            elif isinstance(child, ast.ClassDef):
                visit(child, scopes)   # class bodies do not enclose their methods
            elif isinstance(child, (ast.ListComp, ast.SetComp, ast.DictComp, ast.GeneratorExp)):
                comp = set()
                for gen in child.generators:
                    for t in ast.walk(gen.target):
                        if isinstance(t, ast.Name):
                            comp.add(t.id)
                visit(child, scopes + [comp])
            else:
                if isinstance(child, ast.Name) and isinstance(child.ctx, ast.Load) and len(scopes) > 0:
                    if not any(child.id in s for s in scopes) and child.id not in module_names:
                        problems.append(f"{path}:{child.lineno}: undefined name {child.id!r}")
                visit(child, scopes)

    visit(tree, [])
    return problems


def main():
    files = sys.argv[1:] or (sorted(glob.glob(os.path.join(ROOT, "pbn_rl_amd", "*.py")))
                             + [os.path.join(ROOT, "bench.py"), os.path.join(ROOT, "__graft_entry__.py")]
                             + sorted(glob.glob(os.path.join(ROOT, "tools", "*.py")))
                             + sorted(glob.glob(os.path.join(ROOT, "oracle", "*.py"))))
    problems = []
    for f in files:
        problems += check(f)
    for p in problems:
        print(p)
    sys.exit(1 if problems else 0)


if __name__ == "__main__":
    main()
