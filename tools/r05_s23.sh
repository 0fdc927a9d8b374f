#!/bin/bash
# Round 5 session 23: k_dict_slots on the copy stream from the start (A/B against the previous build,
# alternating, cfg3 and cfg4).
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "200 s23_cfg3 $B --config cfg3" \
  "200 s23_cfg3_base env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg3" \
  "200 s23_cfg4 $B --config cfg4" \
  "200 s23_cfg4_base env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg4" \
  "200 s23_cfg3_b $B --config cfg3" \
  "200 s23_cfg3_base_b env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg3" \
  "200 s23_cfg4_b $B --config cfg4" \
  "200 s23_cfg4_base_b env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg4"
