"""Diagnostic: per-phase cycles of the nested kernels on cfg4 (diag build, PQ_DEBUG_STAMPS=1): k_nest_tile
by default (slots 24-31: its counting half; 32-39: its emission), k_nest_count / k_nest_emit with
PQ_NEST_FUSED=0. The slots are shared with the DELTA walk and the paired dictionary tiles, which cfg4
does not run."""
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

data = workloads.gen_cfg4()[0]
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
print(f"decode {dt*1e3:.3f} ms (cfg4, one decode with stamps)")
tot = sum(int(d[24 + k]) for k in range(8))
fused = os.environ.get("PQ_NEST_FUSED", "1") != "0"
names = (["run_stage", "group_marks", "expansion", "polls(count)", "masks", "lookback+barrier", "validity+publish", "to_lookback"] if fused else
         ["run_stage", "group_marks", "expansion", "page_counts", "packed", "counters", "validity", "-"])
for k, n in enumerate(names):
    v = int(d[24 + k])
    print(f"{'nest_tile ' if fused else 'nest_count'} {n:12s} {v:>16d} cycles (wave sums) {v / max(tot, 1):6.3f}")
tot = sum(int(d[32 + k]) for k in range(8))
for k, n in enumerate(["levels_flags", "entry_index", "offsets", "validity", "groups", "-", "-", "-"]):
    v = int(d[32 + k])
    print(f"{'  (emit)  ' if fused else 'nest_emit '} {n:12s} {v:>16d} cycles (wave sums) {v / max(tot, 1):6.3f}")
