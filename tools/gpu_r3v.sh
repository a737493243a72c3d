#!/bin/bash
# pass V: C5 fp64 queue order: cost classes per doubling of the previous launch's work (Morton cells within)
set -o pipefail
O=gpurun_out/r3v
mkdir -p $O
b() {
  timeout -k 10 400 python -u bench.py --no-cpu --config C5 --steps 2 --warmup 1 "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 $* pero=$RWRT_CELL_PER_OCTAVE', round(d['value']/1e9,4), round(d['ms_per_step'],1), d.get('parity_sample_vs_oracle',{}).get('bitwise'))"
}
RWRT_CELL_PER_OCTAVE=2 b || exit 1
RWRT_CELL_PER_OCTAVE=1 b || exit 1
RWRT_CELL_PER_OCTAVE=4 b || exit 1
RWRT_CELL_PER_OCTAVE=0 b || exit 1
RWRT_CELL_PER_OCTAVE=2 b --probe 12 || exit 1
