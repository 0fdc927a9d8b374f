#!/bin/bash
# the same probe against several library builds (PQGPU_LIB), each process under its own limit
cd "$GRAFT_REPO_ROOT"
V=${VARIANTS:-"[{}]"}
mkdir -p gpurun_out
for lib in ${LIBS:-libpqgpu.so}; do
  for sh in ${SHAPES:-full}; do
    echo "== $lib $sh"
    S=""; [ "$sh" != "full" ] && S="--shape $sh"
    PQGPU_LIB=$PWD/parquet-go-1_amd/lib/$lib timeout -k 10 150 python -u tools/variant_probe.py --config ${CFG:-cfg2} $S --variants "$V" > gpurun_out/lib_$lib_$sh.jsonl 2> gpurun_out/lib.err || { tail -5 gpurun_out/lib.err; exit 1; }
    grep variant gpurun_out/lib_$lib_$sh.jsonl
  done
done
