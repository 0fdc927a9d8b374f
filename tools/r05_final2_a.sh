#!/bin/bash
# Round 5 closing evidence, part A (the build at the end of the round): the -m gpu suite, smoke(), the
# 2-rank rehearsal of the multi-GPU bench path (gloo, both ranks on the one card), and the bench lines
# of cfg1-cfg3 (20 timed steps after 3 warm-ups, with the streamed end-to-end passes and CPU baselines).
cd "$(dirname "$0")/.."
tools/gpu_steps.sh \
  "600 fa2_gpu_all python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 fa2_smoke python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300 fa2_rehearsal_2rank env PQ_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --gather" \
  "300 fa2_bench_cfg1 python -u bench.py --config cfg1 --steps 20 --warmup 3" \
  "300 fa2_bench_cfg2 python -u bench.py --config cfg2 --steps 20 --warmup 3" \
  "300 fa2_bench_cfg3 python -u bench.py --config cfg3 --steps 20 --warmup 3" \
  "300 fa2_verify_cfg4 python -u bench.py --config cfg4 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-e2e" \
  "300 fa2_verify_cfg2 python -u bench.py --config cfg2 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-e2e" \
  "300 fa2_verify_cfg3 python -u bench.py --config cfg3 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-e2e"
