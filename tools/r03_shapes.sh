#!/bin/bash
# cfg2 ablation shapes (tools/variant_probe.py --shape), one process per shape, each under its own limit
cd "$GRAFT_REPO_ROOT"
V=${VARIANTS:-"[{}]"}
mkdir -p gpurun_out
for sh in ${SHAPES:-req plain a b a,req b,req}; do
  echo "== $sh"
  timeout -k 10 120 python -u tools/variant_probe.py --config cfg2 --shape $sh --variants "$V" > gpurun_out/shape_$sh.jsonl 2> gpurun_out/shape_$sh.err || { tail -5 gpurun_out/shape_$sh.err; exit 1; }
  cat gpurun_out/shape_$sh.jsonl
done
