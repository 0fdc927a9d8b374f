"""Diagnostic: per-kernel times of one bench workload with phases removed (diagnostic library,
PQ_ABLATE bits; timing only: outputs are wrong under any ablation).

Bits: 1 k_values no stores, 2 k_values no unpack, 4 k_levels no run expansion, 8 k_levels serial
walk of every run, 256 k_ba_emit no look-back, 512 no pass B, 2048 no length loads, 4096 every
look-back by self-help, 8192 k_ba_emit no payload / offsets stores, 16384 no second slot pieces, 65536 k_nest_emit no offset stores, 131072 no bitmaps, 262144 k_nest_count /
k_nest_emit no level expansion.

usage: python tools/diag_ablate.py cfg2 0,4,8 [rows]
"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PQGPU_LIB", os.path.join(ROOT, "parquet-go-1_amd", "lib", "libpqgpu_diag.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))
import pqgpu  # noqa: E402
from tools import workloads  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
bits = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0").split(",")]
gen = getattr(workloads, "gen_" + cfg)
out = gen(int(sys.argv[3])) if len(sys.argv) > 3 else gen()
data = out[0] if isinstance(out, tuple) else out
ctx = pqgpu.Context(0)
f = pqgpu.File(data)
b = pqgpu.Batch(ctx)
for rg in range(f.num_row_groups):
    for c in range(f.num_columns):
        b.add_file_chunk(f, rg, c)
b.upload()
for ab in bits + [bits[0]]:
    os.environ["PQ_ABLATE"] = str(ab)
    best = {}
    for _ in range(5):
        b.kernel_timing(True)
        b.decode(); b.sync()
        for k, v in b.kernel_times().items():
            best[k] = min(best.get(k, 1e9), v[0])
    print(f"ablate {ab:5d}: " + "  ".join(f"{k} {v:.4f}" for k, v in sorted(best.items())), flush=True)
