"""Schedule / kernel-variant probe: one workload generated once, then decoded by a fresh batch per
variant (environment knobs are read when a batch is created and planned), each timed like bench.py
(warm-up, K timed steps, per-kernel HIP-event medians). One JSON line per variant.

  python tools/variant_probe.py --config cfg2 --variants '[{}, {"PQ_SPEC": "0", "PQ_SPLIT_VALUES": "1"}]'
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402


def cfg2_shape(rows, flags, rg_rows=4_194_304, page_rows=65_536):
    """cfg2's columns with parts of the work removed (probe only): which kernels interfere."""
    import numpy as np
    import pyarrow as pa
    import workloads as W
    rng = np.random.default_rng(2)
    a = np.cumsum(rng.integers(0, 2**16, rows)).astype(np.int64)
    b = rng.random(rows)
    m = None if "req" in flags else rng.random(rows) < 0.1
    m2 = None if "req" in flags else rng.random(rows) < 0.1
    if m is not None:  # no DELTA page with a non-null count = 1 (mod 256) or <= 1 (App. A Q1), as gen_cfg2
        pages = m[: rows // page_rows * page_rows].reshape(-1, page_rows)
        nn = page_rows - pages.sum(1)
        for p in np.flatnonzero((nn % 256 == 1) | (nn <= 1)):
            pages[p, np.flatnonzero(pages[p])[0]] = False
    cols = {}
    if "b" not in flags:
        cols["a"] = pa.array(a, mask=m)
    if "a" not in flags:
        cols["b"] = pa.array(b, mask=m2)
    enc = {k: ("PLAIN" if (k == "b" or "plain" in flags) else "DELTA_BINARY_PACKED") for k in cols}
    return W._write(pa.table(cols), use_dictionary=False, data_page_version="2.0", compression="NONE",
                    column_encoding=enc, max_rows_per_page=page_rows, row_group_size=rg_rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--codec", default="NONE")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--variants", default="[{}]")
    ap.add_argument("--shape", default="", help="cfg2 ablation shapes: req (no nulls), plain (column a PLAIN), "
                                               "a (column a only), b (column b only); comma-separated flags")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    rows = args.rows or cfg["rows"]
    t0 = time.perf_counter()
    if args.shape:
        data = cfg2_shape(rows, set(args.shape.split(",")))
    else:
        data, _ = bench.generate(args.config, rows, 0, args.codec)
    print(json.dumps({"generated_s": round(time.perf_counter() - t0, 1)}), flush=True)
    import pqgpu
    ctx = pqgpu.Context(0)
    f = pqgpu.File(data)
    base_env = dict(os.environ)
    for var in json.loads(args.variants):
        os.environ.clear()
        os.environ.update(base_env)
        os.environ.update({k: str(v) for k, v in var.items()})
        b = pqgpu.Batch(ctx)
        for rg in range(f.num_row_groups):
            for c in range(f.num_columns):
                _, e = b.add_file_chunk(f, rg, c)
                if e is not None:
                    raise e
        b.upload()
        for _ in range(args.warmup):
            b.decode()
        e = b.sync()
        if e is not None:
            raise e
        b.sync()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            b.decode()
        b.sync()
        ms = (time.perf_counter() - t1) / args.steps * 1e3
        kt = bench.kernel_medians(b, max(args.steps, 20))
        st = b.stats()
        print(json.dumps({"variant": var, "ms_per_step": round(ms, 4),
                          "hbm_frac_step": round((st.input_bytes + st.output_bytes) / 1e9 / (ms / 1e3) / 8000.0, 4),
                          "kernels": {k: round(v[0], 4) for k, v in kt.items()}}), flush=True)
        b.close()
    os.environ.clear()
    os.environ.update(base_env)


if __name__ == "__main__":
    main()
