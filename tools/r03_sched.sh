# Schedule experiments for cfg2 (PQ_COPY_MODE etc.); results in gpurun_out/r03/s_<tag>.json
set -e
mkdir -p gpurun_out/r03
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline > gpurun_out/r03/s_$tag.json 2> gpurun_out/r03/s_$tag.err; }
for m in ${MODES:-0 4 5}; do run m$m PQ_COPY_MODE=$m; done
run fused PQ_COPY_FUSED=1
