#!/bin/bash
# Critical path of C3 (zonal and non-zonal) on the current build.
set -o pipefail
mkdir -p gpurun_out/r2c
for bg in zonal nonzonal; do
  timeout -k 10 400 python tools/c4_rehearsal.py --bg $bg --out gpurun_out/r2c/c4_rehearsal_$bg.json > gpurun_out/r2c/c4_$bg.log 2>&1 || { tail -20 gpurun_out/r2c/c4_$bg.log; exit 1; }
  tail -c 600 gpurun_out/r2c/c4_rehearsal_$bg.json
done
