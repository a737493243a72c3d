#!/bin/bash
# pass O: two waves per SIMD (uncached lookups) vs one wave, uncached vs cached
set -o pipefail
O=gpurun_out/r3o
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu --team 0 "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'], d['endpoints_rank0_sha256'])"
}
b --lib rossby-wave-ray-tracing_amd/librwrt_old.so || exit 1
b --lib rossby-wave-ray-tracing_amd/librwrt_2w.so || exit 1
b --lib rossby-wave-ray-tracing_amd/librwrt_nc1w.so || exit 1
b --lib rossby-wave-ray-tracing_amd/librwrt_old.so || exit 1
