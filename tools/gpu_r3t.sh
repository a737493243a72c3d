#!/bin/bash
# pass T: same-build profile summaries for the non-zonal C3 line and the C5 lines (fp64 / fp32
# levels), then each line with its roofline taken from them
set -o pipefail
O=gpurun_out/r3t
mkdir -p $O
run() {   # name, bench args...
  n=$1; shift
  bash tools/profile_round.sh $n "$@" || exit 1
  S=gpurun_out/prof_$n/summary
  timeout -k 10 600 python3 -u bench.py --no-cpu --valu-profile $S/valu.json --traffic $S/traffic.json "$@" > $O/bench_$n.log 2>&1 || { tail $O/bench_$n.log; exit 1; }
  grep '^{' $O/bench_$n.log > $O/bench_$n.json
  python3 -c "import json; d=json.load(open('$O/bench_$n.json')); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], r['bound'], r['frac'], r['profile_same_build'], r.get('valu_issue',{}).get('frac'))"
}
run r3nonzonal --bg nonzonal
run r3c5fp64 --config C5
run r3c5fp32 --config C5 --fields fp32
