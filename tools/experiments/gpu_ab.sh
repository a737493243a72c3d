#!/bin/bash
# A/B of library variants on the C3 bench: tools/gpu_ab.sh <lib> [<lib> ...] (no CPU baseline)
# (BENCH_ARGS overrides the bench arguments, e.g. "--config C5 --fields fp64 --days 10 --steps 2")
set -o pipefail
mkdir -p gpurun_out/ab
args=${BENCH_ARGS:-"--steps 3 --warmup 1"}
for lib in "$@"; do
  n=$(basename $lib .so)
  timeout -k 10 300 python bench.py $args --no-cpu --lib $lib > gpurun_out/ab/$n.log 2>&1 || { tail -5 gpurun_out/ab/$n.log; exit 1; }
  grep -h '^{' gpurun_out/ab/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'])"
done
