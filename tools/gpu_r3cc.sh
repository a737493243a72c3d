#!/bin/bash
# pass CC: write-through (sc1) run-kernel row stores against the default non-temporal ones (A/B, interleaved)
set -o pipefail
O=gpurun_out/r3cc
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['endpoints_rank0_sha256'])"
}
for rep in 1 2 3; do
b || exit 1
b --lib rossby-wave-ray-tracing_amd/librwrt_sc1rows.so || exit 1
done
