#!/bin/bash
# Round 5 session 34: k_nest_tile with the chunks' tiles interleaved in block order (a tile's predecessor
# was dispatched a chunk count of blocks earlier) and 16-B offset stores in the nested emission;
# look-back window back to 16. Full GPU suite, cfg4 benches, nested phase stamps, cfg2.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "400 s34_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s34_cfg4 $B --config cfg4" \
  "200 s34_cfg4_b $B --config cfg4" \
  "200 s34_diag_nest python -u tools/diag_nest.py" \
  "200 s34_tl4 tools/timeline.sh cfg4" \
  "200 s34_cfg2 $B --config cfg2"
# (appended) k_ba_emit pass B with 4 / 8 rounds' slot pieces loaded together (4 waves per SIMD: the
# same two 8-wave workgroups per CU) against the default 2, cfg3
L=parquet-go-1_amd/lib
tools/gpu_steps.sh \
  "200 s34_cfg3 $B --config cfg3" \
  "200 s34_cfg3_bag4 env PQGPU_LIB=$L/libpqgpu_bag4.so $B --config cfg3" \
  "200 s34_cfg3_bag8 env PQGPU_LIB=$L/libpqgpu_bag8.so $B --config cfg3" \
  "200 s34_cfg3_b $B --config cfg3"
