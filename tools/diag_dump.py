"""Diagnostic: every phase-stamp counter slot of one decode (PQ_DEBUG_STAMPS=1, libpqgpu_diag.so).

usage: python tools/diag_dump.py <cfg> [rows]   -> slot, total cycles (nonzero slots only). Slot bases:
0 list-ranking levels / k_levels_bw1, 16 k_levels_seg(w), 32 k_level_fill, 40 k_ba_emit (47: waves),
48 hyb_scan in k_levels_hyb / k_snappy, 56 hyb_scan in k_scan_runs, 8 DELTA values.
"""
import os
import sys
os.environ["PQ_DEBUG_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PQGPU_LIB", os.path.join(ROOT, "parquet-go-1_amd", "lib", "libpqgpu_diag.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))
import pqgpu  # noqa: E402
from tools import workloads  # noqa: E402

cfg = sys.argv[1]
rows = int(sys.argv[2]) if len(sys.argv) > 2 else None
out = getattr(workloads, "gen_" + cfg)(rows) if rows else getattr(workloads, "gen_" + cfg)()
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
b.decode(); b.sync()
d = b.debug_counters()
for k in range(64):
    if int(d[k]):
        print(f"slot {k:2d} {int(d[k]):>16d}")
