"""Page-index result visibility experiment.

Builds the device page index of a few fixtures `--builds` times each, in ONE process, and counts per
build the re-reads the host needed (polls), the chunks whose completion marker never arrived
(unreported) and the chunks that fell back. Prints one JSON line. Round 3 ran it under two scratch /
fence knobs (PQ_IX_POOL=1: scratch from hipMallocAsync's pool; PQ_IX_FENCE=1: system-scope release
fences around the walk's result stores; profiles/r03_ix_visibility_experiment.jsonl); round 5
removed both from the library, so today it measures the product configuration only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pqgpu  # noqa: E402
import pqtest  # noqa: E402


def main():
    builds = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    names = ["cfg5_small", "types_v1", "cfg2_v2_small", "cfg4_small", "cfg1"]
    ctx = pqgpu.Context(0)
    out = {"env": {k: os.environ[k] for k in ("PQ_IX_POOL", "PQ_IX_FENCE") if k in os.environ}, "builds": 0,
           "polls": 0, "unreported": 0, "fallback_chunks": 0, "builds_with_unreported": 0, "per_fixture": {}}
    for name in names:
        try:
            data = pqtest.load(name)
        except Exception:
            continue
        f = pqgpu.File(data)
        chunks = [(rg, c) for rg in range(f.num_row_groups) for c in range(f.num_columns)]
        ref = None
        agg = {"builds": 0, "polls": 0, "unreported": 0, "mismatch": 0}
        for _ in range(builds):
            ix = pqgpu.PageIndex.for_chunks(ctx, f, chunks, whole_file=True)
            st = ix.stats()
            res = [ix.chunk(k) for k in range(len(chunks))]
            if ref is None:
                ref = res
            agg["builds"] += 1
            agg["polls"] += st["polls"]
            agg["unreported"] += st["unreported"]
            agg["mismatch"] += int(res != ref and st["unreported"] == 0)
            out["builds"] += 1
            out["polls"] += st["polls"]
            out["unreported"] += st["unreported"]
            out["fallback_chunks"] += st["fallback_chunks"]
            out["builds_with_unreported"] += int(st["unreported"] > 0)
            ix.close()
        out["per_fixture"][name] = agg
    # concurrent builds: the streaming pipeline's worker threads build the indexes of different row
    # groups at once, each on its own slot stream (the configuration of the original failures)
    for name in ("cfg5_small", "cfg2_v2_small", "cfg4_small"):
        try:
            data = pqtest.load(name)
        except Exception:
            continue
        f = pqgpu.File(data)
        rgs = list(range(f.num_row_groups)) * max(1, 64 // max(1, f.num_row_groups))
        p = pqgpu.Pipeline(ctx, f, row_groups=rgs, depth=8, threads=8, device_index=True)
        fails = 0
        for _rg, _b, err in p:
            fails += err is not None
        st = p.stats()
        p.close()
        out["per_fixture"][name + "_pipeline"] = {"row_groups": len(rgs), "polls": st["ix_polls"],
                                                  "unreported": st["ix_unreported"],
                                                  "fallback_chunks": st["ix_fallback_chunks"], "failed_row_groups": fails}
        out["polls"] += st["ix_polls"]
        out["unreported"] += st["ix_unreported"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
