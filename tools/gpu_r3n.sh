#!/bin/bash
# pass N: lead launches then time-budgeted phases (experiment)
set -o pipefail
O=gpurun_out/r3n
mkdir -p $O
b() {
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'], d['endpoints_rank0_sha256'])"
}
b --bg nonzonal || exit 1
b --bg nonzonal --phases t:40,40,40 --team 0 || exit 1
b --bg nonzonal --phases t:25,25,25,25,25 --team 0 || exit 1
b --bg nonzonal --phases t:40,40,40 --team 128 || exit 1
b || exit 1
b --team 128 || exit 1
b --phases t:40,40,40 --team 0 || exit 1
b --phases t:40,40,40 --team 128 || exit 1
