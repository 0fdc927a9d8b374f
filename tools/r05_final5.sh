#!/bin/bash
# Round 5: the committed build after the SWAR level expansion and compress16 -- GPU suite, smoke(),
# default bench line (cfg2), cfg4's full bench line and full-size verification, then cfg4's rocprofv3
# evidence (kernel trace + stats, FETCH_SIZE, WRITE_SIZE, SQ; tools/prof.sh via tools/evidence.sh).
cd "$(dirname "$0")/.."
tools/gpu_steps.sh \
  "600 f5_gpu_all python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 f5_smoke python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300 f5_bench_default python -u bench.py" \
  "300 f5_bench_cfg4 python -u bench.py --config cfg4 --steps 20 --warmup 3" \
  "300 f5_verify_cfg4 python -u bench.py --config cfg4 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-e2e" \
  "600 f5_prof python -u -c 'import subprocess,sys; sys.exit(subprocess.call([\"tools/evidence.sh\",\"cfg4\"]))'"
