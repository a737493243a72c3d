#!/bin/bash
# Launch-length sweep of the C3 bench (tail vs cost-prediction staleness).
set -o pipefail
mkdir -p gpurun_out/chunks
for bg in nonzonal zonal; do
for c in 0 480 240 120; do
  timeout -k 10 200 python bench.py --bg $bg --chunk $c --steps 3 --warmup 1 --no-cpu > gpurun_out/chunks/${bg}_$c.log 2>&1 || { tail -5 gpurun_out/chunks/${bg}_$c.log; exit 1; }
  grep -h '^{' gpurun_out/chunks/${bg}_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$bg', $c, d['value'], d['ms_per_step'], d['config']['launch_rows'])"
done; done
