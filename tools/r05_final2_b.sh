#!/bin/bash
# Round 5 closing evidence, part B: the bench lines of cfg4 / cfg5, then tools/prof.sh per workload
# (rocprofv3 kernel trace + stats, FETCH_SIZE, WRITE_SIZE and SQ passes, each its own run under its own
# limit).
cd "$(dirname "$0")/.."
tools/gpu_steps.sh \
  "300 fb2_bench_cfg4 python -u bench.py --config cfg4 --steps 20 --warmup 3" \
  "400 fb2_bench_cfg5 python -u bench.py --config cfg5 --steps 20 --warmup 3" \
  "800 fb2_prof python -u -c 'import subprocess,sys; sys.exit(subprocess.call([\"tools/evidence.sh\",\"cfg1\",\"cfg2\",\"cfg3\",\"cfg4\",\"cfg5\"]))'"
