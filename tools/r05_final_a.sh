#!/bin/bash
# Round 5 evidence, part A: the -m gpu suite, smoke(), the 2-rank rehearsal of the multi-GPU bench path
# (gloo, both ranks on the one card), and the bench lines of cfg1-cfg3 (20 timed steps after 3 warm-ups,
# with the streamed end-to-end passes and the CPU baselines).
cd "$(dirname "$0")/.."
tools/gpu_steps.sh \
  "600 fa_gpu_all python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 fa_smoke python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "300 fa_rehearsal_2rank env PQ_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --gather" \
  "300 fa_bench_cfg1 python -u bench.py --config cfg1 --steps 20 --warmup 3" \
  "300 fa_bench_cfg2 python -u bench.py --config cfg2 --steps 20 --warmup 3" \
  "300 fa_bench_cfg3 python -u bench.py --config cfg3 --steps 20 --warmup 3"
