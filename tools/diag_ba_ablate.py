"""Diagnostic: k_ba_emit time with phases removed (diagnostic library, PQ_ABLATE bits):
256 no look-back (base 0), 512 no pass B, 2048 no length loads, 4096 every look-back by
self-help. Timing only: outputs are wrong under any ablation.

usage: python tools/diag_ba_ablate.py [cfg3]
"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PQGPU_LIB", os.path.join(ROOT, "parquet-go-1_amd", "lib", "libpqgpu_diag.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))
import pqgpu  # noqa: E402
from tools import workloads  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
out = getattr(workloads, "gen_" + cfg)()
data = out[0] if isinstance(out, tuple) else out
ctx = pqgpu.Context(0)
f = pqgpu.File(data)
b = pqgpu.Batch(ctx)
for rg in range(f.num_row_groups):
    for c in range(f.num_columns):
        b.add_file_chunk(f, rg, c)
b.upload()
for ab in [0, 256, 512, 256 | 512, 2048, 2048 | 256 | 512, 0]:
    os.environ["PQ_ABLATE"] = str(ab)
    ms = []
    for _ in range(5):
        b.kernel_timing(True)
        b.decode(); b.sync()
        kt = b.kernel_times()
        ms.append(sum(v[0] for k, v in kt.items() if "emit" in k))
    print(f"ablate {ab:5d}: k_ba_emit* {min(ms):.4f} ms (min of 5) {[round(x, 4) for x in ms]}", flush=True)
