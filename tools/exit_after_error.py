"""Regression check: a process that raises with a live Context and Batch (the traceback keeps
them alive) must exit with the Python error status, not crash in teardown."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-go-1_amd")]
import pqgpu  # noqa: E402

ctx = pqgpu.Context(0)
b = pqgpu.Batch(ctx)
f = pqgpu.File(open(os.path.join(ROOT, "tests", "golden", "cfg1.parquet"), "rb").read())
cid, e = b.add_file_chunk(f, 0, 0)
b.decode()
b.sync()
raise RuntimeError("deliberate error with live handles")
