#!/bin/bash
# A/B timing of kernel build variants on the GPU box (one bench line each).
# usage: tools/experiments/ab_variants.sh <tag> <days> [extra bench args]
tag=$1; days=$2; shift 2
mkdir -p gpurun_out
for lib in rossby-wave-ray-tracing_amd/librwrt_*.so; do
  for order in ${ORDERS:-cost}; do
    timeout -k 10 300 python bench.py --days "$days" --steps 2 --warmup 1 --no-cpu --lib "$lib" --order "$order" "$@" \
      >> gpurun_out/ab_${tag}.jsonl 2>> gpurun_out/ab_${tag}.err || { echo "FAILED $lib $order"; exit 1; }
  done
done
