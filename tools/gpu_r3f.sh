#!/bin/bash
set -o pipefail
for bg in nonzonal zonal; do
BG=$bg bash tools/gpu_sched_sweep.sh "" "--first-chunk 24,160,80,360 --order total" "--first-chunk 24,160,170,270 --order total" "--first-chunk 24,160,300 --order total" "--first-chunk 24,160,80,360" || exit 1
done
