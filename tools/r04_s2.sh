#!/bin/bash
# Round-4 session 2: the whole -m gpu suite, configs[4] as specified (1e9 rows, 256 row groups, N=1,
# sampled verification), cfg2 copy/occupancy variants, evidence for cfg5 and cfg1.
cd "$(dirname "$0")/.."
L=$PWD/parquet-go-1_amd/lib
exec tools/gpu_steps.sh \
  "400 gpu_tests python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "600 strong_cfg5 python -u bench.py --config cfg5 --strong --verify --verify-every 16" \
  "200 probe_cfg2 python -u tools/variant_probe.py --config cfg2 --variants '[{}, {\"PQ_COPY_FUSED\": \"0\"}, {\"PQ_DELTA_TILED\": \"1\"}]'" \
  "150 probe_cfg2_cu8 env PQGPU_LIB=$L/libpqgpu_cu8.so python -u tools/variant_probe.py --config cfg2 --variants '[{}]'" \
  "150 probe_cfg2_wpe6 env PQGPU_LIB=$L/libpqgpu_wpe6.so python -u tools/variant_probe.py --config cfg2 --variants '[{}]'" \
  "400 bench_cfg5 python -u bench.py --config cfg5 --steps 20 --warmup 3" \
  "700 prof_cfg5 tools/prof.sh cfg5" \
  "300 bench_cfg1 python -u bench.py --config cfg1 --steps 20 --warmup 3" \
  "400 prof_cfg1 tools/prof.sh cfg1" \
  "$@"
