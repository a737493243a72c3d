#!/bin/bash
# pass EE: the cell cache's 24 LDS reads per lookup in 2 or 3 groups (RWRT_CACHE_READ_GROUPS;
# VGPR spills to AGPRs 158 -> 8) against all 24 in flight at once (default), interleaved
set -o pipefail
O=gpurun_out/r3ee
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['endpoints_rank0_sha256'], d['library_sha256'])"
}
L=rossby-wave-ray-tracing_amd
for rep in 1 2 3; do
b || exit 1
b --lib $L/librwrt_g2.so || exit 1
b --lib $L/librwrt_g3.so || exit 1
done
for rep in 1 2; do
b --bg nonzonal || exit 1
b --bg nonzonal --lib $L/librwrt_g2.so || exit 1
b --bg nonzonal --lib $L/librwrt_g3.so || exit 1
done
