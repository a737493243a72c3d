#!/bin/bash
# pass FF: the grouped cell-cache reads without the scheduling barrier between a group's reads
# and its blends (RWRT_CACHE_GROUP_FREE=1; 2, 3 or 6 groups) against the default (2 groups, barrier)
set -o pipefail
O=gpurun_out/r3ff
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['endpoints_rank0_sha256'], d['library_sha256'])"
}
L=rossby-wave-ray-tracing_amd
for rep in 1 2 3; do
b || exit 1
b --lib $L/librwrt_f2.so || exit 1
b --lib $L/librwrt_f3.so || exit 1
b --lib $L/librwrt_f6.so || exit 1
done
