#!/bin/bash
# End-of-round GPU pass on the committed tree: GPU suite, smoke, profile summaries of
# this build (rocprof stats + traffic + VALU), then the driver's bench command.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
bash tools/profile_round.sh r2final || exit 1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_final.log 2>&1 || { tail gpurun_out/bench_final.log; exit 1; }
grep '^{' gpurun_out/bench_final.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['profile_same_build'], d.get('bitwise_vs_cpu_oracle',{}).get('identical_values_frac'))"
