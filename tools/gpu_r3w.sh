#!/bin/bash
# pass W: C3 probe / lead-launch lengths with the per-launch latency mode default
set -o pipefail
O=gpurun_out/r3w
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'], d['endpoints_rank0_sha256'])"
}
for rep in 1 2; do
b || exit 1
b --probe 4 || exit 1
b --first-chunk 24,128 || exit 1
b --first-chunk 24,192 || exit 1
b --first-chunk 32,160 || exit 1
b --team 64,384,64 || exit 1
done
