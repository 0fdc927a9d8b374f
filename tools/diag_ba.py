"""Diagnostic: per-phase cycle counters of k_ba_emit on a bench workload (PQ_DEBUG_STAMPS=1).

usage: python tools/diag_ba.py [cfg3] [rows]   (needs `make diag` -> lib/libpqgpu_diag.so)
"""
import os
import sys
import time
os.environ["PQ_DEBUG_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PQGPU_LIB", os.path.join(ROOT, "parquet-go-1_amd", "lib", "libpqgpu_diag.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))
import pqgpu  # noqa: E402
from tools import workloads  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else None
gen = getattr(workloads, "gen_" + cfg)
out = gen(rows) if rows else gen()
data = out[0] if isinstance(out, tuple) else out
ctx = pqgpu.Context(0)
f = pqgpu.File(data)
b = pqgpu.Batch(ctx)
for rg in range(f.num_row_groups):
    for c in range(f.num_columns):
        b.add_file_chunk(f, rg, c)
b.upload()
b.decode(); b.sync()
b.debug_counters(reset=True)
t0 = time.perf_counter()
b.decode(); b.sync()
dt = time.perf_counter() - t0
d = b.debug_counters()
tiles = int(d[47])
print(f"decode {dt*1e3:.3f} ms; k_ba_emit waves {tiles}")
for k, n in enumerate(["draw+tile_load", "passA", "barrier1", "lookback(w0)", "barrier2", "passB", "lb_windows#"]):
    v = int(d[40 + k])
    print(f"emit {n:16s} total {v:>14d}  per wave {v / max(tiles, 1):>12.1f}")
