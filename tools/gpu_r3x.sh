#!/bin/bash
# pass X: the non-zonal line under the new defaults (4-row probe, latency mode 64/256/64) vs round-2's
set -o pipefail
O=gpurun_out/r3x
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu --bg nonzonal "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('BENCH nonzonal $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'], d['endpoints_rank0_sha256'], r['frac'], r['profile_same_build'])"
}
for rep in 1 2; do
b || exit 1
b --probe 6 --team 0 || exit 1
b --probe 6 || exit 1
done
