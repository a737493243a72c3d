#!/bin/bash
# Profile summaries of the current build (rocprof stats + FETCH/WRITE + SQ VALU passes of the C3
# bench), then the driver's bench command, which picks those summaries up (same library sha).
set -o pipefail
mkdir -p gpurun_out
bash tools/profile_round.sh "$1" || exit 1
ls gpurun_out/prof_$1/summary
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$1.log 2>&1 || { tail gpurun_out/bench_$1.log; exit 1; }
grep '^{' gpurun_out/bench_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['profile_same_build'], r['valu_source'], d.get('bitwise_vs_cpu_oracle',{}).get('identical_values_frac'))"
