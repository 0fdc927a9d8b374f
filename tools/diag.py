"""Diagnostic: per-phase cycle counters of k_levels and the DELTA values path (PQ_DEBUG_STAMPS=1)."""
import os
import sys
import time
os.environ["PQ_DEBUG_STAMPS"] = "1"
os.environ.setdefault("PQGPU_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "parquet-go-1_amd", "lib", "libpqgpu_diag.so"))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))
import pqgpu  # noqa: E402
from tools import workloads  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].isdigit() else "cfg2"
args = [a for a in sys.argv[1:] if a.isdigit()]
rows = int(args[0]) if args else None
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
pages = f.num_row_groups * 64 * 2
print(f"decode {dt*1e3:.3f} ms ({cfg}); per-page figures assume cfg2's {pages} level pages")
names = ["stage", "P1_links", "P2_doubling", "P3_ckp", "P4_walkers", "P5_P6", "tail", "chunk_top"]
for k, n in enumerate(names):
    v = int(d[k])
    print(f"levels {n:12s} total {v:>14d}  per page(wave) {v / pages / 4:>12.1f}")
for k, nm in enumerate(["seg_stage", "seg_A", "seg_B", "seg_CD", "seg_store", "seg_B_iters", "seg_A_steps", "seg_D_steps"]):
    v = int(d[16 + k])
    print(f"levels {nm:12s} total {v:>14d}  per page(wave) {v / pages:>12.1f}")
for k, nm in enumerate(["w_first", "w_fetch_issue", "w_walk", "w_bar1", "w_store", "w_bar2", "w_reloads#", "w_windows#"]):
    v = int(d[24 + k])
    print(f"dwalk  {nm:12s} total {v:>14d}  per page(wave) {v / (pages // 2) / 4:>12.1f}")
dn = ["reload", "walk_wait", "unpack", "scan", "write", "hops#x4", "parse", "walk_w0"]
for k, n in enumerate(dn):
    v = int(d[8 + k])
    print(f"delta  {n:12s} total {v:>14d}  per page(wave) {v / (pages // 2) / 4:>12.1f}")
dd = ["load", "indices", "stores_issue", "drain", "waves#"]
nw = max(1, int(d[36]))
for k, n in enumerate(dd):
    v = int(d[32 + k])
    print(f"dict2  {n:12s} total {v:>14d}  per wave {v / nw:>12.1f}")
sn = ["fast_hops", "decode", "chain", "sink", "window", "hops#", "steps#", "-"]
for k, n in enumerate(sn[:7]):
    v = int(d[56 + k])
    print(f"scan   {n:12s} total {v:>14d}")
for k, n in enumerate(sn[:7]):  # k_levels_hyb's hyb_scan (slots 48..; k_snappy's too where it runs)
    v = int(d[48 + k])
    print(f"lvhyb  {n:12s} total {v:>14d}")
