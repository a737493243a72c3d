#!/bin/bash
# pass U: latency mode per launch (the 160-row launch is bound by its heaviest rays' chains)
set -o pipefail
O=gpurun_out/r3u
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'], d['endpoints_rank0_sha256'])"
}
for rep in 1 2; do
b --team 0 || exit 1
b --team 0,256,0 || exit 1
b --team 0,512,0 || exit 1
b --team 64,256,64 || exit 1
b --team 0,1024,0 || exit 1
done
