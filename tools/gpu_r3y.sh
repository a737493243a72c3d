#!/bin/bash
# pass Y: same-build profile of the non-zonal line under its defaults (4-row probe, no latency mode)
set -o pipefail
O=gpurun_out/r3y
mkdir -p $O
bash tools/profile_round.sh r3nonzonal2 --bg nonzonal || exit 1
S=gpurun_out/prof_r3nonzonal2/summary
for rep in 1 2; do
timeout -k 10 300 python3 -u bench.py --no-cpu --bg nonzonal --valu-profile $S/valu.json --traffic $S/traffic.json > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench_nonzonal_$rep.json
python3 -c "import json; d=json.load(open('$O/bench_nonzonal_$rep.json')); r=d['roofline']; print('nonzonal', d['value'], d['ms_per_step'], d['config']['launch_rows'], r['frac'], r['profile_same_build'])"
done
