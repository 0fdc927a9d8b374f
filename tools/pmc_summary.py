"""Summarise tools/pmc_traffic.sh output: per decode kernel (k_values dispatches split into
the DELTA and the other work-item launches by launch order), the average FETCH_SIZE and
WRITE_SIZE per launch, the gfx950-corrected HBM bytes (FETCH_SIZE reads 1/2 of a wide
coalesced streaming read on gfx950, MI355X_MICROARCH.md §HBM: doubled) and the kernel-trace
average duration. Writes profiles/<name>.json (read by bench.py for roofline.traffic)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


SPLIT = os.environ.get("PQ_SPLIT_VALUES") == "1"


def kname(name, order):
    if "k_values" in name:
        if not SPLIT:
            return "k_values"
        return "k_values[delta]" if order % 2 == 0 else "k_values[other]"
    if "k_levels" in name:
        return "k_levels"
    return name


def counters(path, counter):
    rows = list(csv.DictReader(open(path)))
    per = defaultdict(float)  # dispatch -> value (sum over XCD/SE instances)
    names = {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        per[d] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    out = defaultdict(list)
    seen = defaultdict(int)
    for d in sorted(per):
        base = "k_values" if "k_values" in names[d] else names[d]
        out[kname(names[d], seen[base])].append(per[d])
        seen[base] += 1
    return out


def main(src, name):
    f = counters(glob.glob(os.path.join(src, "fetch", "**", "*counter_collection.csv"), recursive=True)[0], "FETCH_SIZE")
    w = counters(glob.glob(os.path.join(src, "write", "**", "*counter_collection.csv"), recursive=True)[0], "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fk = sum(f[k]) / len(f[k]) if f[k] else 0.0
        wk = sum(w[k]) / len(w[k]) if w[k] else 0.0
        res[k] = {"launches": len(f[k]), "FETCH_SIZE_KiB": round(fk, 1), "WRITE_SIZE_KiB": round(wk, 1),
                  "hbm_bytes_raw": int((fk + wk) * 1024), "hbm_bytes_corrected": int((2 * fk + wk) * 1024)}
    trace = glob.glob(os.path.join(src, "stats", "**", "*kernel_trace.csv"), recursive=True)
    if trace:  # per-dispatch durations, k_values split by launch order like the counters
        dur = defaultdict(list)
        seen = defaultdict(int)
        rows = sorted(csv.DictReader(open(trace[0])), key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            nm = r["Kernel_Name"]
            if "k_values" not in nm and "k_levels" not in nm:
                continue
            base = "k_values" if "k_values" in nm else nm
            dur[kname(nm, seen[base])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            seen[base] += 1
        for k, v in dur.items():
            if k in res:
                res[k]["trace_avg_us"] = round(sum(v) / len(v), 2)
                res[k]["trace_dispatches"] = len(v)
    out = {"source": "tools/pmc_traffic.sh (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
           "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads, MI355X_MICROARCH.md HBM section)",
           "command": "python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline", "kernels": res}
    path = os.path.join(ROOT, "profiles", name + ".json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc_traffic"),
         sys.argv[2] if len(sys.argv) > 2 else "r01_pmc_traffic")
