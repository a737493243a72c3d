#!/bin/bash
# latency-mode size sweep on the zonal C3 bench (one GPU)
set -o pipefail
O=gpurun_out/team_sweep
mkdir -p $O
for t in auto 0 64 256 1024; do
  timeout -k 10 300 python -u bench.py --no-cpu --team $t > $O/t$t.log 2>&1 || { tail -5 $O/t$t.log; exit 1; }
  grep '^{' $O/t$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('team $t', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['endpoints_rank0_sha256'])"
done
