#!/bin/bash
# Round 5 session 36: k_nest_tile with two tiles per workgroup (both tiles counted and their aggregates
# published before either looks back) against one (libpqgpu_t1); full GPU suite; phase stamps with the
# look-back round trips; cfg5 kernel timeline.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "400 s36_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s36_cfg4 $B --config cfg4" \
  "200 s36_cfg4_t1 env PQGPU_LIB=$L/libpqgpu_t1.so $B --config cfg4" \
  "200 s36_cfg4_b $B --config cfg4" \
  "200 s36_cfg4_t1_b env PQGPU_LIB=$L/libpqgpu_t1.so $B --config cfg4" \
  "200 s36_diag_nest python -u tools/diag_nest.py" \
  "300 s36_tl5 tools/timeline.sh cfg5"
