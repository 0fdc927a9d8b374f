"""Diagnostic: k_snappy phase cycles per page (PQ_DEBUG_STAMPS=1, diagnostic library) for the
snappy_probe page contents: element decode, chain follow, batch execution, long literals.
usage: python tools/diag_snappy.py [int64_small|double_optional|double_required]"""
import os
import sys
import time
os.environ["PQ_DEBUG_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PQGPU_LIB", os.path.join(ROOT, "parquet-go-1_amd", "lib", "libpqgpu_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pqgpu  # noqa: E402
import snappy_probe as S  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "int64_small"
data = S.make(kind)
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
pages = b.stats().snappy_pages
print(f"{kind}: decode {dt*1e3:.3f} ms, {pages} SNAPPY pages")
for k, n in enumerate(["decode", "chain", "batch", "long_lit", "windows#", "elements#", "batch_bytes#", "tail"]):
    v = int(d[48 + k])
    print(f"snappy {n:13s} total {v:>14d}  per page {v / max(pages, 1):>14.1f}")
