"""bench.py — decoded-output throughput of the MI355X Parquet column-chunk decoder.

Workload (BASELINE.json configs[1], "cfg2"): INT64 DELTA_BINARY_PACKED +
DOUBLE PLAIN columns, 67,108,864 rows in 16 row groups of 4,194,304 rows,
OPTIONAL with 10% nulls (RLE def levels), data page V2 (65,536 rows per
page), UNCOMPRESSED; synthetic data (numpy default_rng seeds 2 and 3) written
by pyarrow, Q1-safe (no DELTA page with NN ≡ 1 mod 256).

A "step" decodes every column chunk of every row group once (levels ->
validity bitmaps, DELTA prefix sums, PLAIN copies) with the pages already
resident in HBM. Multi-GPU: each rank decodes its own cfg2-sized shard of row
groups (weak scaling, no collective on the data path); the launcher contract
is in the task description (torch.distributed.run, one rank per GPU).

Prints ONE JSON line (rank 0) with value = decoded-output GB/s over all
ranks, plus the roofline of the dominant kernel (HIP events on its stream)
and the CPU baseline (the oracle, a value-at-a-time C restatement of the
reference decoders, timed on this host's cores).
"""
import argparse
import ctypes
import io
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md


def gen_cfg2(rows=67_108_864, rg_rows=4_194_304, page_rows=65_536, seed=2, first_rg=0, codec="NONE"):
    """cfg2 file bytes: row groups [first_rg, first_rg + rows / rg_rows) of one
    logical file whose row group g is drawn from default_rng([seed, g]) (column a) and
    default_rng([seed + 1, g]) (column b), so rank shards are a row-group partition of one file.
    Null masks are nudged so that no DELTA page has a non-null count ≡ 1 (mod 256) or ≤ 1
    (Appendix A Q1: the reference fails on those)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    nrg = max(1, -(-rows // rg_rows))
    parts = []
    for g in range(first_rg, first_rg + nrg):
        n = min(rg_rows, rows - (g - first_rg) * rg_rows)
        rng = np.random.default_rng([seed, g])
        rng3 = np.random.default_rng([seed + 1, g])
        # column a: running sum of uniform [0, 2^16) increments, restarted per row group at
        # g * 2^15 * rg_rows (its expected start), so row group g is the same in every shard
        parts.append((np.cumsum(rng.integers(0, 2**16, n)) + g * 2**15 * rg_rows, rng.random(n) < 0.1,
                      rng3.random(n), rng3.random(n) < 0.1))
    a = np.concatenate([p[0] for p in parts]).astype(np.int64)
    m = np.concatenate([p[1] for p in parts])
    b = np.concatenate([p[2] for p in parts])
    m2 = np.concatenate([p[3] for p in parts])
    pages = m[: rows // page_rows * page_rows].reshape(-1, page_rows)
    nn = page_rows - pages.sum(1)
    for p in np.flatnonzero((nn % 256 == 1) | (nn <= 1)):
        k = np.flatnonzero(pages[p])[0]
        pages[p, k] = False  # one more non-null value
    t = pa.table({"a": pa.array(a, mask=m), "b": pa.array(b, mask=m2)})
    bio = io.BytesIO()
    # SNAPPY pages are V1 (cfg5's page version): pyarrow stores an incompressible V2 values
    # section uncompressed with is_compressed=false, which the reference ignores (page_v2.go:125)
    pq.write_table(t, bio, use_dictionary=False, data_page_version="2.0" if codec == "NONE" else "1.0",
                   compression=codec,
                   column_encoding={"a": "DELTA_BINARY_PACKED", "b": "PLAIN"}, max_rows_per_page=page_rows,
                   row_group_size=rg_rows, write_statistics=False)
    return bio.getvalue(), (a, m, b, m2)


def cpu_baseline(data, budget_s=20.0, codec="NONE"):
    """The oracle (CPU port of the reference decoders) on this host: one thread per chunk,
    threads = min(16, cores). Returns (rows/s, GB/s decoded output, threads, sample description)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import py_oracle as O
    f = O.File(data)
    chunks = [(rg, c) for rg in range(f.num_row_groups) for c in range(f.num_columns)]
    threads = max(1, min(16, os.cpu_count() or 1))
    # probe one chunk to size the sample to the budget
    t0 = time.perf_counter()
    f.read_chunk(*chunks[0])
    per_chunk = time.perf_counter() - t0
    n = int(max(threads, min(len(chunks), budget_s * threads / max(per_chunk, 1e-6))))
    n = min(n, len(chunks))
    sample = chunks[:n]
    out_bytes = [0]
    rows = [0]
    lock = threading.Lock()
    it = iter(sample)

    def work():
        while True:
            with lock:
                try:
                    rg, c = next(it)
                except StopIteration:
                    return
            r = f.read_chunk(rg, c)
            with lock:
                out_bytes[0] += r.num_values * 8 + (len(r.def_levels) + 7) // 8
                rows[0] += len(r.def_levels) / f.num_columns

    t0 = time.perf_counter()
    ts = [threading.Thread(target=work) for _ in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    desc = (f"{n} of {len(chunks)} column chunks ({n * 4194304 // 2 / 1e6:.0f}M rows x col) of cfg2"
            + ("" if codec == "NONE" else f" ({codec} pages, decompressed by the oracle)") + ", oracle liboracle.so")
    return rows[0] / dt, out_bytes[0] / dt / 1e9, threads, desc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=67_108_864)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--codec", choices=["NONE", "SNAPPY"], default="NONE",
                    help="SNAPPY: the same cfg2 file with SNAPPY pages, decompressed on the device "
                         "(k_snappy) inside every step (cfg5's codec; not the headline line)")
    ap.add_argument("--verify", action="store_true", help="check every decoded value against the generator")
    ap.add_argument("--gather", action="store_true",
                    help="N>1: after the timed decode, all-gather column a over RCCL into one contiguous "
                         "column on every rank and time it separately (SURVEY §8(e), optional)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = 0
    red_dev = "cuda"
    if world > 1:
        import torch
        import torch.distributed as dist
        # one rank per GPU; PQ_BENCH_BACKEND=gloo (with ranks sharing a card) only rehearses the
        # multi-rank path on a 1-GPU box: timing then reduces on the CPU
        backend = os.environ.get("PQ_BENCH_BACKEND", "nccl")
        device = local_rank % torch.cuda.device_count()
        torch.cuda.set_device(device)  # torch initialises HIP before libpqgpu loads (one runtime)
        torch.zeros(1, device=f"cuda:{device}")
        dist.init_process_group(backend)
        red_dev = "cuda" if backend == "nccl" else "cpu"
    import pqgpu
    from pqgpu import shard

    # weak scaling: the logical file has 16 row groups of cfg2 per GPU; rank r decodes its
    # contiguous row-group range (no collective on the data path)
    rg_rows = 4_194_304
    per_rank_rg = max(1, -(-args.rows // rg_rows))
    g0, g1 = shard.row_group_range(per_rank_rg * world, rank, world)
    data, truth = gen_cfg2(min(args.rows, (g1 - g0) * rg_rows), rg_rows=rg_rows, first_rg=g0, codec=args.codec)
    ctx = pqgpu.Context(device)
    f = pqgpu.File(data)
    b = pqgpu.Batch(ctx)
    ids = []
    for rg in range(f.num_row_groups):
        for c in range(f.num_columns):
            cid, e = b.add_file_chunk(f, rg, c)
            if e is not None:
                raise e
            ids.append(cid)
    b.upload()
    for _ in range(args.warmup):
        b.decode()
    e = b.sync()
    if e is not None:
        raise e
    if args.verify:
        a, m, bb, m2 = truth
        per = args.rows // f.num_row_groups if f.num_row_groups else 0
        for k, cid in enumerate(ids):
            rg, c = divmod(k, 2)
            r = b.result(cid)
            sl = slice(rg * per, (rg + 1) * per)
            src, msk = (a, m) if c == 0 else (bb.view(np.uint64), m2)
            assert np.array_equal(r.values_raw, src[sl][~msk[sl]]), f"verify failed rg{rg} col{c}"
            assert np.array_equal(r.validity_bits(), (~msk[sl]).astype(np.uint8)), f"validity rg{rg} col{c}"

    def barrier():
        if dist is not None:
            dist.barrier()
        b.sync()

    b.kernel_timing(True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.decode()
    b.sync()
    barrier()
    dt = time.perf_counter() - t0
    st = b.stats()
    kern_ms, kern_n, kern_name = b.kernel_time()
    ktimes = b.kernel_times()
    dt = shard.max_over_ranks(dt, dist, device=red_dev)
    ms_per_step = dt / args.steps * 1e3
    rows_total = args.rows * world
    out_gb = st.output_bytes * world / 1e9
    algo_bytes = st.input_bytes + st.output_bytes  # per rank, per step
    value = out_gb / (ms_per_step / 1e3)
    rows_per_s = rows_total / (ms_per_step / 1e3)

    # roofline of the dominant kernel: algorithmic bytes moved by that kernel per launch / its avg time
    kb = kernel_bytes(b, kern_name, st) or 0
    achieved = kb / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else 0.0
    traffic, traffic_src = pmc_traffic(kern_name, args.rows, os.path.join(
        ROOT, "profiles", "r01_pmc_traffic.json" if args.codec == "NONE" else "r01_s7_pmc_snappy.json"))
    line = {
        "metric": "decoded GB/s + rows/s per GPU and whole node (1/2/4/8); % HBM peak",
        "value": round(value, 2),
        "unit": "GB/s (decoded output)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64+f64 (bit copies), u8 levels",
        "data": "synthetic (numpy default_rng([2|3, row group]); pyarrow 25 writer)",
        "config": {"workload": "cfg2: INT64 DELTA_BINARY_PACKED + DOUBLE PLAIN, OPTIONAL 10% nulls, "
                               + ("V2, UNCOMPRESSED" if args.codec == "NONE" else
                                  "V1, SNAPPY (pages resident compressed, decompressed on the device every step)"), "rows_per_gpu": args.rows, "row_groups_per_gpu": f.num_row_groups,
                   "page_rows": 65536, "parallelism": f"row-group shards x{world}"},
        "rows_per_s": round(rows_per_s, 1),
        "algorithmic_GBps": round(algo_bytes * world / 1e9 / (ms_per_step / 1e3), 2),
        "hbm_frac_step": round(algo_bytes / 1e9 / (ms_per_step / 1e3) / HBM_PEAK_GBS, 4),
        "bytes_per_step": {"input": st.input_bytes, "output": st.output_bytes},
        "roofline": {"bound": "hbm", "kernel": kern_name, "kernel_ms": round(kern_ms, 4),
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_src, "bytes_per_launch": kb},
        "kernels": {k: {"ms": round(ms, 4), "launches_per_step": round(n / args.steps, 2),
                        "GBps": round(kernel_bytes(b, k, st) / (ms / 1e3) / 1e9, 1)
                        if kernel_bytes(b, k, st) is not None and ms > 0 else None}
                    for k, (ms, n) in ktimes.items()},
    }
    if args.gather and dist is not None:
        import torch
        col_a = shard.device_values(b, ids[0::2], f"cuda:{device}")
        if red_dev == "cpu":  # gloo rehearsal: gather host copies
            col_a = col_a.cpu()
        shard.gather_column(col_a, dist)  # warm-up (communicator setup)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        whole = shard.gather_column(col_a, dist)
        torch.cuda.synchronize()
        gdt = shard.max_over_ranks(time.perf_counter() - t0, dist, device=red_dev)
        line["allgather"] = {"column": "a", "bytes_per_rank": col_a.numel() * 8,
                             "bytes_out": whole.numel() * 8, "ms": round(gdt * 1e3, 3),
                             "GBps_out": round(whole.numel() * 8 / gdt / 1e9, 1), "backend": dist.get_backend()}
    if rank == 0 and not args.no_cpu_baseline:
        rps, gbs, thr, desc = cpu_baseline(data, codec=args.codec)
        line["cpu_baseline"] = {"value": round(gbs, 3), "unit": "GB/s (decoded output)", "rows_per_s": round(rps, 1),
                                "cores": thr, "kind": "port", "sample": desc,
                                "host_cpus": os.cpu_count()}
    if rank == 0:
        print(json.dumps(line))
    b.close()
    if dist is not None:
        dist.destroy_process_group()


def pmc_traffic(kernel, rows, path=os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")):
    """HBM bytes per launch of `kernel` from the committed PMC run of this same workload
    (tools/pmc_traffic.sh + tools/pmc_summary.py: FETCH_SIZE / WRITE_SIZE in separate passes,
    FETCH_SIZE doubled per the gfx950 calibration). rocprofv3 cannot run inside the bench
    process, so the counters come from that run; None when absent or for another workload."""
    if rows != 67_108_864 or not os.path.exists(path):
        return None, None
    k = json.load(open(path))["kernels"].get(kernel)
    if not k:
        return None, None
    return k["hbm_bytes_corrected"], os.path.relpath(path, ROOT)


def kernel_bytes(b, name, st):
    """Algorithmic bytes of one launch of kernel `name` (SURVEY §8(d) accounting restricted to what
    that kernel reads and writes): k_values = value sections read + values written; k_levels =
    rep/def sections read + validity bitmap / levels written."""
    if name == "k_values[delta]":
        return int(st.delta_kernel_bytes)
    if name == "k_values[other]":
        return int(st.values_kernel_bytes - st.delta_kernel_bytes)
    if name == "k_values":  # DELTA and the other value work items in one launch
        return int(st.values_kernel_bytes)
    if name == "k_levels":
        return int(st.levels_kernel_bytes)
    if name == "k_snappy":
        return int(st.snappy_kernel_bytes)
    return None


if __name__ == "__main__":
    main()
