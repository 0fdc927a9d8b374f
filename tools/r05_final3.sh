#!/bin/bash
# Round 5: the committed build at the round's end -- GPU suite, smoke(), default bench line (cfg2) and
# cfg4 (k_nest_tcount present, off), full-size cfg4 verification.
cd "$(dirname "$0")/.."
tools/gpu_steps.sh \
  "600 f3_gpu_all python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 f3_smoke python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300 f3_bench_default python -u bench.py" \
  "300 f3_bench_cfg4 python -u bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e" \
  "300 f3_verify_cfg4 python -u bench.py --config cfg4 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-e2e"
