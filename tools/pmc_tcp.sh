#!/bin/bash
# One rocprofv3 --pmc pass of L1 / L2 request counters for a bench workload (is a kernel bound by
# L2 -> L1 line traffic?): TCP_TCC_READ_REQ (L1 misses sent to L2), TCP_TOTAL_CACHE_ACCESSES,
# TCP_PENDING_STALL_CYCLES, TA_BUSY, TCC_HIT / TCC_MISS. Summary: tools/pmc_sum.py-style per kernel.
# usage: tools/pmc_tcp.sh <config> [extra bench args]  -> gpurun_out/tcp_<config>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
CFG=${1:-cfg3}; shift
OUT=gpurun_out/tcp_$CFG
mkdir -p $OUT
CMD="python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-e2e $*"
P="TCP_TCC_READ_REQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum,TCP_PENDING_STALL_CYCLES_sum,TA_BUSY_avr,TCC_HIT_sum,TCC_MISS_sum"
timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc -o run -- $CMD > $OUT/pmc.log 2>&1
rc=$?
tail -n 3 $OUT/pmc.log
[ $rc -ne 0 ] && exit $rc
python3 - "$OUT" <<'PY'
import csv, glob, sys, json
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True)[0]
per = defaultdict(lambda: defaultdict(float)); names = {}
for r in csv.DictReader(open(f)):
    d = int(r["Dispatch_Id"]); per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    names[d] = r["Kernel_Name"].split("(")[0].split("::")[-1]
agg = defaultdict(lambda: defaultdict(list))
for d, cs in per.items():
    for c, v in cs.items(): agg[names[d]][c].append(v)
out = {k: {c: round(sum(v) / len(v)) for c, v in cs.items()} | {"dispatches": len(next(iter(cs.values())))} for k, cs in agg.items()}
json.dump(out, open(sys.argv[1] + "/tcp_summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
