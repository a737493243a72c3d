#!/bin/bash
# pass GG: what the latency mode's code in the run kernel costs the ray loop -- a build
# without it (RWRT_NOQUAD=1: SGPR spill slots 222 -> 157) against the default, both with
# no rays in latency mode (--team 0), interleaved
set -o pipefail
O=gpurun_out/r3gg
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['endpoints_rank0_sha256'], d['library_sha256'])"
}
L=rossby-wave-ray-tracing_amd
for rep in 1 2 3; do
b --team 0 || exit 1
b --team 0 --lib $L/librwrt_noquad.so || exit 1
done
b --team 0 --bg nonzonal || exit 1
b --team 0 --bg nonzonal --lib $L/librwrt_noquad.so || exit 1
