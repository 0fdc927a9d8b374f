#!/bin/bash
# Round 5: the committed build at the round's end (after the s41-s45 probes, all reverted; new
# back-to-back nested tests) -- GPU suite, smoke(), default bench line (cfg2), cfg4 and cfg3 lines,
# full-size cfg4 verification.
cd "$(dirname "$0")/.."
tools/gpu_steps.sh \
  "600 f4_gpu_all python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 f4_smoke python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300 f4_bench_default python -u bench.py" \
  "300 f4_bench_cfg4 python -u bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e" \
  "300 f4_bench_cfg3 python -u bench.py --config cfg3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e" \
  "300 f4_verify_cfg4 python -u bench.py --config cfg4 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-e2e"
