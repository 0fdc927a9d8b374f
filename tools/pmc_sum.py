"""Per-kernel sums of a rocprofv3 counter_collection.csv (tools/pmc_pass.sh output), per dispatch.
usage: python tools/pmc_sum.py gpurun_out/pmc_cfg4_insts [kernel-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("pq::", "")
    if want not in k:
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, v in sorted(agg.items()):
    n = max(1, len(disp[k]))
    print(f"{k[:32]:32s} x{n:<3d} " + "  ".join(f"{c.replace('SQ_', '')}={x / n:.4g}" for c, x in sorted(v.items())))
