#!/bin/bash
# Round-end evidence on one GPU: the -m gpu suite, a 2-rank rehearsal of the multi-GPU bench path
# (gloo, both ranks on the one card), then rocprofv3 kernel stats + PMC passes per config.
cd "$(dirname "$0")/.."
tools/gpu_steps.sh \
  "600 gpu_all python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "300 rehearsal_2rank env PQ_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --gather" \
  "300 rehearsal_2rank_strong env PQ_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --config cfg5 --strong --total-rgs 16 --no-cpu-baseline --verify" || exit $?
grep -q " passed" gpurun_out/gpu_all.log && ! grep -q "failed" gpurun_out/gpu_all.log || exit 1
[ -n "$EVIDENCE" ] && tools/evidence.sh $EVIDENCE
exit 0
