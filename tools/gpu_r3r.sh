#!/bin/bash
# pass R: C4 rehearsal (one set split over W ranks, each shard timed alone) with the latency mode
# choosing 16 rays per wave (default) or also 4 per wave
set -o pipefail
O=gpurun_out/r3r
mkdir -p $O
timeout -k 10 500 python -u tools/c4_rehearsal.py --worlds 1,8 --out $O/c4_d16.json > $O/c4_d16.log 2>&1 || { tail -5 $O/c4_d16.log; exit 1; }
grep world $O/c4_d16.log
RWRT_QUAD_DENSITIES=4,16 timeout -k 10 500 python -u tools/c4_rehearsal.py --worlds 1,8 --out $O/c4_d4.json > $O/c4_d4.log 2>&1 || { tail -5 $O/c4_d4.log; exit 1; }
grep world $O/c4_d4.log
