#!/bin/bash
# Round 5 session 35: k_nest_tile's look-back -- round trips per tile (diagnostic build), and polling
# without s_sleep against the default; cfg5 kernel timeline.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "200 s35_diag_nest python -u tools/diag_nest.py" \
  "200 s35_cfg4 $B --config cfg4" \
  "200 s35_cfg4_nosleep env PQGPU_LIB=$L/libpqgpu_nosleep.so $B --config cfg4" \
  "200 s35_cfg4_b $B --config cfg4" \
  "200 s35_cfg4_nosleep_b env PQGPU_LIB=$L/libpqgpu_nosleep.so $B --config cfg4" \
  "300 s35_tl5 tools/timeline.sh cfg5"
