#!/bin/bash
# Round 5 session 30: nested batches with k_nest_pcount (page counts from the run tables, k_bases no
# longer waits for the nested arrays) + k_nest_tile on the aux stream + repetition-stream level kernels
# beside the definition streams'; k_ba_emit with first pieces in pass A by default. Full GPU suite,
# cfg4 A/B of the schedule switches, cfg3 default; cfg2 priority probes of the level kernel.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "400 s30_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s30_cfg4 $B --config cfg4" \
  "200 s30_cfg4_nopcount env PQ_NEST_PCOUNT=0 $B --config cfg4" \
  "200 s30_cfg4_nosplit env PQ_LV_SPLIT=0 $B --config cfg4" \
  "200 s30_cfg4_presum0 env PQ_BA_PRESUM=0 $B --config cfg4" \
  "200 s30_cfg4_b $B --config cfg4" \
  "200 s30_tl4 tools/timeline.sh cfg4" \
  "200 s30_cfg3 $B --config cfg3" \
  "200 s30_cfg2 $B --config cfg2" \
  "200 s30_cfg2_segp2 env PQGPU_LIB=$L/libpqgpu_segp2.so $B --config cfg2" \
  "200 s30_cfg2_segp3 env PQGPU_LIB=$L/libpqgpu_segp3.so $B --config cfg2" \
  "200 s30_cfg2_dsprio env PQ_DELTA_STREAM_PRIO=1 $B --config cfg2" \
  "200 s30_cfg2_b $B --config cfg2"
