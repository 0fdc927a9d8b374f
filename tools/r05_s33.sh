#!/bin/bash
# Round 5 session 33: BatchDev zero-initialised (an uninitialised err_next let the serial re-decode's
# k_values_delta wipe a key buffer: bad_def_empty_run lost its error); k_nest_tile look-back window 64
# predecessors (against 16); full GPU suite; cfg2 / cfg4 benches; nested phase stamps.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "400 s33_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s33_cfg4 $B --config cfg4" \
  "200 s33_cfg4_win16 env PQGPU_LIB=$L/libpqgpu_win16.so $B --config cfg4" \
  "200 s33_cfg4_b $B --config cfg4" \
  "200 s33_diag_nest python -u tools/diag_nest.py" \
  "200 s33_cfg2 $B --config cfg2" \
  "200 s33_cfg3 $B --config cfg3"
