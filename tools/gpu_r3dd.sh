#!/bin/bash
# pass DD: C5 fp64 -- the upper level's corner gathers issued before the wait on the
# lower level's LDS-DMA refill (RWRT_C5_UPPER_EARLY=1) against the default (A/B, interleaved)
set -o pipefail
O=gpurun_out/r3dd
mkdir -p $O
b() {
  timeout -k 10 400 python -u bench.py --no-cpu --config C5 "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['parity_sample_vs_oracle']['bitwise'], d['library_sha256'])"
}
for rep in 1 2; do
b || exit 1
b --lib rossby-wave-ray-tracing_amd/librwrt_c5early.so || exit 1
done
