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


def _bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True, text=True,
                       timeout=timeout, cwd="/tmp")
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, lines, p.stderr


def test_bench_gpus_flag_starts_the_ranks():
    """`bench.py --gpus 2` without a launcher starts two ranks itself (torch.distributed.run, gloo here)
    and each decodes its own contiguous row-group shard: [0, 16) and [16, 32) of cfg2's 32 (weak
    scaling, 16 per GPU). The SCALE run cannot silently measure one rank."""
    rc, lines, err = _bench(["--gpus", "2", "--plan"], {"PQ_BENCH_BACKEND": "gloo"})
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, lines
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["backend"] == "gloo"
    assert [s["row_groups"] for s in ln["shards"]] == [[0, 16], [16, 32]]


def test_bench_refuses_a_world_size_other_than_gpus():
    """Under a launcher whose WORLD_SIZE is not --gpus, bench.py exits non-zero and prints no line."""
    rc, lines, err = _bench(["--gpus", "1", "--plan"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert rc != 0 and not lines and "WORLD_SIZE" in err
    rc, lines, _ = _bench(["--gpus", "1", "--plan"])
    assert rc == 0 and lines[0]["n_gpus"] == 1 and lines[0]["shards"] == [{"rank": 0, "row_groups": [0, 16]}]
