"""k_snappy cost by page content: decode time of SNAPPY V1 files whose pages are (1) one
incompressible DOUBLE stream (long literals only), (2) the same column OPTIONAL (a def-level
bitmap of ~1,500 short elements ahead of the literals), (3) a compressible INT64 column
(short copies throughout). Prints one JSON line per case."""
import io
import json
import os
import sys

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))
import pqgpu  # noqa: E402

ROWS, RG, PAGE = 16 * 1048576, 4194304, 65536


def make(kind):
    rng = np.random.default_rng(7)
    if kind == "double_required":
        t = pa.table({"b": pa.array(rng.random(ROWS))})
    elif kind == "double_optional":
        t = pa.table({"b": pa.array(rng.random(ROWS), mask=rng.random(ROWS) < 0.1)})
    else:
        t = pa.table({"c": pa.array(rng.integers(0, 16, ROWS).astype(np.int64))})
    bio = io.BytesIO()
    pq.write_table(t, bio, use_dictionary=False, data_page_version="1.0", compression="SNAPPY",
                   column_encoding={t.column_names[0]: "PLAIN"}, max_rows_per_page=PAGE, row_group_size=RG,
                   write_statistics=False)
    return bio.getvalue()


def main():
    ctx = pqgpu.Context(0)
    for kind in ("double_required", "double_optional", "int64_small"):
        data = make(kind)
        f = pqgpu.File(data)
        b = pqgpu.Batch(ctx)
        for rg in range(f.num_row_groups):
            _, e = b.add_file_chunk(f, rg, 0)
            assert e is None, e
        b.upload()
        b.decode()
        assert b.sync() is None
        b.kernel_timing(True)
        for _ in range(10):
            b.decode()
        b.sync()
        kt = b.kernel_times()
        st = b.stats()
        print(json.dumps({"case": kind, "pages": int(st.snappy_pages), "file_MB": round(len(data) / 1e6, 1),
                          "k_snappy_ms": round(kt["k_snappy"][0], 4),
                          "k_snappy_GBps": round(st.snappy_kernel_bytes / kt["k_snappy"][0] / 1e6, 1)}), flush=True)
        b.close()


if __name__ == "__main__":
    main()
