#!/bin/bash
# pass P: non-zonal C3 with the heaviest rays of every launch in latency mode (quad_rays)
set -o pipefail
O=gpurun_out/r3p
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'], d['endpoints_rank0_sha256'])"
}
b --bg nonzonal --team 0 || exit 1
b --bg nonzonal --team 64 || exit 1
b --bg nonzonal --team 128 || exit 1
b --bg nonzonal --team 256 || exit 1
b --bg nonzonal --team 512 || exit 1
b --bg nonzonal --team 128 --first-chunk 24,160,300,300 || exit 1
b --bg nonzonal --team 0 || exit 1
b --team 0 || exit 1
b --team 64 || exit 1
