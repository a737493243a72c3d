#!/bin/bash
# pass BB: same-build profile summaries (non-temporal row stores build) for the non-zonal C3 line
# and the C5 lines, each line then run with them
set -o pipefail
O=gpurun_out/r3bb
mkdir -p $O
run() {   # name, bench args...
  n=$1; shift
  bash tools/profile_round.sh $n "$@" || exit 1
  S=gpurun_out/prof_$n/summary
  timeout -k 10 600 python3 -u bench.py --no-cpu --valu-profile $S/valu.json --traffic $S/traffic.json "$@" > $O/bench_$n.log 2>&1 || { tail $O/bench_$n.log; exit 1; }
  grep '^{' $O/bench_$n.log > $S/bench_line.json
  python3 -c "import json; d=json.load(open('$S/bench_line.json')); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], r['bound'], r['frac'], r['profile_same_build'], r.get('valu_issue',{}).get('frac'))"
}
run r3bbnonzonal --bg nonzonal
run r3bbc5fp64 --config C5
run r3bbc5fp32 --config C5 --fields fp32
