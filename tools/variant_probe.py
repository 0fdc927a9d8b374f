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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--codec", default="NONE")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--variants", default="[{}]")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    rows = args.rows or cfg["rows"]
    t0 = time.perf_counter()
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
