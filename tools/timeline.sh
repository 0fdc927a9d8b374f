#!/bin/bash
# Kernel timeline of a few bench steps (rocprofv3 --kernel-trace): which launches overlap.
# usage: tools/timeline.sh <config> [extra bench args]  -> gpurun_out/tl_<config>/timeline.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
CFG=${1:-cfg2}; shift
OUT=gpurun_out/tl_$CFG
mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-e2e "$@" > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python3 - "$OUT" <<'PY' | tee $OUT/timeline.txt
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"]]
# the timed loop's steps (untimed launches; the bench's per-kernel event pass comes after them): a
# step starts with the launch that started the first (warm-up) step; print timed steps 1 and 2
names = [r["Kernel_Name"].split("(")[0].split("::")[-1] for r in rows]
grid = lambda r: int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
r0 = next((i for i, n in enumerate(names) if n == "k_reset"), 0)
steps = [i for i in range(len(rows)) if names[i] == names[r0] and grid(rows[i]) == grid(rows[r0])]
tail = rows[steps[1]:steps[3]] if len(steps) >= 4 else rows[-40:]
t0 = int(tail[0]["Start_Timestamp"])
for r in tail:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{r['Kernel_Name'].split('(')[0].split('::')[-1]:22s} grid {int(r.get('Grid_Size', r.get('Grid_Size_X', 0)) or 0):>9} "
          f"wg {r.get('Workgroup_Size', r.get('Workgroup_Size_X', '')):>5} start {s/1e3:9.1f} us  end {e/1e3:9.1f} us  dur {(e-s)/1e3:8.1f} us")
PY
