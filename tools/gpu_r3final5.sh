#!/bin/bash
# Round-3 final pass 5 (cell-cache reads in two groups): GPU suite, smoke, same-build
# profile of the default bench command, then the driver's bench command.
set -o pipefail
O=gpurun_out/r3final5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
grep -E "passed|failed" $O/pytest_gpu.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile_round.sh r3final5 || exit 1
S=gpurun_out/prof_r3final5/summary
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --valu-profile $S/valu.json --traffic $S/traffic.json > $O/bench_driver_cmd.log 2>&1 || { tail $O/bench_driver_cmd.log; exit 1; }
grep '^{' $O/bench_driver_cmd.log > $O/bench_driver_cmd.json
python3 -c "import json; d=json.load(open('$O/bench_driver_cmd.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('profile_same_build'), d.get('bitwise_vs_cpu_oracle',{}).get('identical_values_frac'))"
# the other lines' same-build profiles (as tools/gpu_r3bb.sh)
run() {   # name, bench args...
  n=$1; shift
  bash tools/profile_round.sh $n "$@" || exit 1
  S=gpurun_out/prof_$n/summary
  timeout -k 10 600 python3 -u bench.py --no-cpu --valu-profile $S/valu.json --traffic $S/traffic.json "$@" > $O/bench_$n.log 2>&1 || { tail $O/bench_$n.log; exit 1; }
  grep '^{' $O/bench_$n.log > $S/bench_line.json
  python3 -c "import json; d=json.load(open('$S/bench_line.json')); r=d['roofline']; print('$n', d['value'], d['ms_per_step'], r['bound'], r['frac'], r['profile_same_build'], r.get('valu_issue',{}).get('frac'))"
}
run r3f5nonzonal --bg nonzonal
run r3f5c5fp64 --config C5
run r3f5c5fp32 --config C5 --fields fp32
