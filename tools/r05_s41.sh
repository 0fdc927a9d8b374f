#!/bin/bash
# Round 5 session 41: cfg2 with the DELTA page waves at issue priority 1 / 2 outside their walk
# (PQ_DELTA_PRIO; the fused copies stay at 0) against the default 0, alternating.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg2"
tools/gpu_steps.sh \
  "200 s41_cfg2 $B" \
  "200 s41_cfg2_dp1 env PQGPU_LIB=$L/libpqgpu_dp1.so $B" \
  "200 s41_cfg2_dp2 env PQGPU_LIB=$L/libpqgpu_dp2.so $B" \
  "200 s41_cfg2_b $B" \
  "200 s41_cfg2_dp1_b env PQGPU_LIB=$L/libpqgpu_dp1.so $B" \
  "200 s41_cfg2_dp2_b env PQGPU_LIB=$L/libpqgpu_dp2.so $B" \
  "200 s41_cfg5 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg5" \
  "200 s41_cfg5_dp2 env PQGPU_LIB=$L/libpqgpu_dp2.so python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg5"
