#!/bin/bash
# pass Q: C5 (0.25 deg, 90 d, BASELINE size) launch length with the cost x Morton-cell queue order
set -o pipefail
O=gpurun_out/r3q
mkdir -p $O
b() {
  timeout -k 10 400 python -u bench.py --no-cpu --config C5 --steps 2 --warmup 1 "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'][:4], len(d['config']['launch_rows']), d.get('parity_sample_vs_oracle',{}).get('bitwise', d.get('parity_sample_vs_oracle')))"
}
b || exit 1
b --chunk 32 || exit 1
b --chunk 72 || exit 1
b --chunk 96 || exit 1
b --first-chunk 24 || exit 1
b --fields fp32 || exit 1
b --fields fp32 --chunk 120 || exit 1
