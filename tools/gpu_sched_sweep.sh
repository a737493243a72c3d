#!/bin/bash
# Work-queue order / launch schedule sweep of the C3 bench (one line each).
#   BG=nonzonal tools/gpu_sched_sweep.sh "<bench args>" "<bench args>" ...
set -o pipefail
O=gpurun_out/sched_${BG:-nonzonal}
mkdir -p $O
k=0
for cfg in "$@"; do
  k=$((k+1))
  timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 --bg ${BG:-nonzonal} $cfg > $O/run$k.log 2>&1 || { tail -5 $O/run$k.log; exit 1; }
  grep '^{' $O/run$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg |', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'], d['endpoints_rank0_sha256'])"
done
