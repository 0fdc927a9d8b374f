"""Summarise tools/prof.sh output into profiles/<round>_pmc_<config>.json: per kernel the
kernel-trace average duration, FETCH_SIZE / WRITE_SIZE per launch (FETCH_SIZE doubled: gfx950
wide streaming reads count half, MI355X_MICROARCH.md §HBM), the corrected HBM bytes, and the SQ
counters (waves, stall buckets, LDS bank-conflict cycles / LDS cycles). bench.py reads
`hbm_bytes_corrected` of its dominant kernel as roofline.traffic.
usage: python tools/prof_summary.py <config> [round]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


SLOT_KERNELS = {  # bench / library timer slot -> the kernels it brackets
    "k_ba_emit": ["k_ba_emit", "k_ba_emit_slots", "k_ba_emit_slots64", "k_ba_emit_lds"],
    "k_levels": ["k_levels", "k_levels_bw1", "k_levels_seg", "k_levels_segw", "k_levels_hyb", "k_levels_bw1w", "k_levels_w"],
    "k_values_delta": ["k_values_delta"],
    "k_values_dict": ["k_values_dict", "k_values_dict2"],
}


def short(name):
    n = name.split("(")[0].split("<")[0]
    for p in ("pq::", "void "):
        n = n.replace(p, "")
    return n.strip()


def per_dispatch(path):
    """{counter: {kernel: [value per dispatch]}} (values summed over XCD / SE instances)."""
    acc = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        acc[(r["Counter_Name"], d)] += float(r["Counter_Value"])
        names[d] = short(r["Kernel_Name"])
    out = defaultdict(lambda: defaultdict(list))
    for (c, d), v in sorted(acc.items(), key=lambda x: x[0][1]):
        out[c][names[d]].append(v)
    return out


def main(cfg, rnd="r02"):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{cfg}")
    res = defaultdict(dict)
    trace = glob.glob(os.path.join(src, "stats", "**", "*kernel_trace.csv"), recursive=True)
    if trace:
        dur = defaultdict(list)
        for r in csv.DictReader(open(trace[0])):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k, v in dur.items():
            res[k]["trace_avg_us"] = round(sum(v) / len(v), 2)
            res[k]["trace_dispatches"] = len(v)
    for sub in ("fetch", "write", "sq"):
        f = glob.glob(os.path.join(src, sub, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        for c, ks in per_dispatch(f[0]).items():
            for k, v in ks.items():
                res[k][c] = round(sum(v) / len(v), 1)
    for k, r in res.items():
        if "FETCH_SIZE" in r or "WRITE_SIZE" in r:
            fk, wk = r.get("FETCH_SIZE", 0.0), r.get("WRITE_SIZE", 0.0)
            r["hbm_bytes_raw"] = int((fk + wk) * 1024)
            r["hbm_bytes_corrected"] = int((2 * fk + wk) * 1024)
        if r.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_bank_conflict_frac"] = round(r.get("SQ_LDS_BANK_CONFLICT", 0) / r["SQ_LDS_IDX_ACTIVE"], 4)
        if r.get("SQ_WAVE_CYCLES") and r.get("trace_avg_us"):
            # SQ_WAVE_CYCLES counts quad-cycles of resident waves: mean resident waves per CU
            # at the clock the chip holds (~2.1 GHz under load assumed)
            r["mean_waves_per_cu"] = round(4 * r["SQ_WAVE_CYCLES"] / (r["trace_avg_us"] * 1e-6 * 2.1e9) / 256, 2)
        if r.get("SQ_WAVE_CYCLES"):
            w = r["SQ_WAVE_CYCLES"]
            r["stall_frac"] = {"wait_any": round(r.get("SQ_WAIT_ANY", 0) / w, 3),
                               "wait_inst_any": round(r.get("SQ_WAIT_INST_ANY", 0) / w, 3),
                               "active_inst_any": round(r.get("SQ_ACTIVE_INST_ANY", 0) / w, 3)}
    # the stats pass's own bench line: its roofline kernel's live HIP-event mean against the trace
    line, check = None, None
    log = os.path.join(src, "stats.log")
    if os.path.exists(log):
        for ln in open(log):
            if ln.startswith("{") and '"roofline"' in ln:
                line = json.loads(ln)
    if line:
        rf = line["roofline"]
        k = rf["kernel"]
        # a timer slot may cover several kernels launched one after the other on its stream
        ks = [x for x in SLOT_KERNELS.get(k, [k]) if x in res and "trace_avg_us" in res[x]]
        steps = line["warmup"] + line["steps"] + max(line["steps"], 20)  # + bench.kernel_means' steps
        if ks:
            tot_us = sum(res[x]["trace_avg_us"] * res[x]["trace_dispatches"] for x in ks)
            tr_ms = tot_us / 1e3 / steps
            frac_tr = rf["bytes_per_launch"] * rf.get("launches_per_step", 1) / (tr_ms / 1e3) / 1e9 / rf["peak"]
            check = {"kernel": k, "trace_kernels": ks, "line_kernel_ms": rf["kernel_ms"], "line_frac": rf["frac"],
                     "trace_ms_per_step": round(tr_ms, 4), "trace_frac": round(frac_tr, 4),
                     "line_over_trace": round(rf["kernel_ms"] / tr_ms, 4),
                     "note": f"trace: the kernels' summed durations over every step of the command ({steps}: "
                             "warm-up, timed and bench.kernel_means' steps)"}
    stats = glob.glob(os.path.join(src, "stats", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        import shutil
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{rnd}_{cfg}_kernel_stats.csv"))
    out = {"source": "tools/prof.sh (rocprofv3: kernel trace; --pmc FETCH_SIZE, WRITE_SIZE and 8 SQ counters, "
                     "separate passes)", "config": cfg,
           "command": f"python3 bench.py --config {cfg} --steps 20 --warmup 3 --no-cpu-baseline --no-e2e",
           "bench_line": line, "line_vs_trace": check,
           "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads, MI355X_MICROARCH.md HBM section)",
           "kernels": res}
    path = os.path.join(ROOT, "profiles", f"{rnd}_pmc_{cfg}.json")
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(*sys.argv[1:])
