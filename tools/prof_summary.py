"""Summarise a rocprofv3 kernel trace (SQLite .db or *_kernel_stats.csv / *_kernel_trace.csv) per kernel."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    q = ("select name, count(*), avg(duration), min(duration), max(duration), sum(duration), max(grid_x), "
         "max(workgroup_x), max(vgpr_count), max(sgpr_count), max(lds_size), max(scratch_size) "
         "from kernels group by name order by sum(duration) desc")
    return list(c.execute(q))


def from_trace_csv(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        k = r["Kernel_Name"]
        e = rows.setdefault(k, [k, 0, 0, 1 << 62, 0, 0, 0, 0, 0, 0, 0, 0])
        e[1] += 1
        e[5] += d
        e[3] = min(e[3], d)
        e[4] = max(e[4], d)
        e[6] = max(e[6], int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0))
        e[7] = max(e[7], int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0))
        e[8] = max(e[8], int(r.get("VGPR_Count", 0) or 0))
        e[9] = max(e[9], int(r.get("SGPR_Count", 0) or 0))
        e[10] = max(e[10], int(r.get("LDS_Block_Size", r.get("Lds_Size", 0)) or 0))
        e[11] = max(e[11], int(r.get("Scratch_Size", 0) or 0))
    out = []
    for e in rows.values():
        e[2] = e[5] / e[1]
        out.append(tuple(e))
    return sorted(out, key=lambda x: -x[5])


def main(path):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        csvs = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = (csvs or dbs)[0]
    rows = from_db(path) if path.endswith(".db") else from_trace_csv(path)
    print(f"# source: {os.path.basename(path)} (durations in microseconds)")
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'total_us':>11s} "
          f"{'grid':>8s} {'wg':>4s} {'vgpr':>5s} {'sgpr':>5s} {'lds':>6s} {'scratch':>7s}")
    for r in rows:
        name = r[0].split("(")[0][:60]
        print(f"{name:60s} {r[1]:6d} {r[2] / 1e3:10.2f} {r[3] / 1e3:10.2f} {r[4] / 1e3:10.2f} {r[5] / 1e3:11.1f} "
              f"{r[6]:8d} {r[7]:4d} {r[8]:5d} {r[9]:5d} {r[10]:6d} {r[11]:7d}")


if __name__ == "__main__":
    main(sys.argv[1])
