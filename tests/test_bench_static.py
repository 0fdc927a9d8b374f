"""bench.py on the CPU: every name its functions call is defined (the GPU legs never run here, so a
helper lost in an edit would only show on the box), and the e2e window arithmetic."""
import ast
import builtins
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_calls_only_defined_names():
    src = open(os.path.join(ROOT, "bench.py")).read()
    t = ast.parse(src)
    defined = {n.name for n in ast.walk(t) if isinstance(n, (ast.FunctionDef, ast.ClassDef))}
    defined |= {a.asname or a.name.split(".")[0] for n in ast.walk(t) if isinstance(n, (ast.Import, ast.ImportFrom))
                for a in n.names}
    defined |= {n.id for n in ast.walk(t) if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Store)}
    defined |= {n.arg for n in ast.walk(t) if isinstance(n, ast.arg)}
    called = {n.func.id for n in ast.walk(t) if isinstance(n, ast.Call) and isinstance(n.func, ast.Name)}
    missing = sorted(c for c in called if c not in defined and not hasattr(builtins, c))
    assert not missing, missing
