#!/bin/bash
# pass S: C3 lead-launch schedules (one lead launch instead of 24 + 160), two repetitions
set -o pipefail
O=gpurun_out/r3s
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'], d['endpoints_rank0_sha256'])"
}
for rep in 1 2; do
b || exit 1
b --first-chunk 184 || exit 1
b --first-chunk 24,160,446 || exit 1
b --first-chunk 90 || exit 1
b --first-chunk 24,360 || exit 1
done
