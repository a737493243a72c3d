#!/bin/bash
# A/B timing matrix on the GPU box: one bench line per "lib|bench args" entry.
# usage: tools/experiments/ab_matrix.sh <tag> "librwrt.so|--chunk 55" "librwrt_w2g2.so|--chunk 1080" ...
tag=$1; shift
mkdir -p gpurun_out
for cfg in "$@"; do
  lib=rossby-wave-ray-tracing_amd/${cfg%%|*}; args=${cfg#*|}
  echo "== $cfg" >> gpurun_out/ab_${tag}.err
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --lib "$lib" $args \
    >> gpurun_out/ab_${tag}.jsonl 2>> gpurun_out/ab_${tag}.err || { echo "FAILED $cfg"; exit 1; }
done
