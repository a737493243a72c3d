#!/bin/bash
# A/B of library variants on the C3 bench: tools/gpu_ab.sh <lib> [<lib> ...] (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out/ab
for lib in "$@"; do
  n=$(basename $lib .so)
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --lib $lib > gpurun_out/ab/$n.log 2>&1 || { tail -5 gpurun_out/ab/$n.log; exit 1; }
  grep -h '^{' gpurun_out/ab/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'])"
done
