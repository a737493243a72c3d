#!/bin/bash
# Round 3, pass D: RK4 90-day C3 tests, per-row cost capture, schedule sweep
# (non-zonal C3), cell-ordered queue on C5.
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3_ref90.py -x -v --timeout 300 --timeout-method thread > $O/pytest_ref90.log 2>&1 || { tail -30 $O/pytest_ref90.log; exit 1; }
grep -E "passed|failed" $O/pytest_ref90.log | tail -1
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench_zonal.log 2>&1 || { tail -5 $O/bench_zonal.log; exit 1; }
grep '^{' $O/bench_zonal.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3 zonal', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['endpoints_rank0_sha256'], d['library_sha256'])"
mkdir -p gpurun_out/rowcost
timeout -k 10 400 python -u tools/c3_row_costs.py --out gpurun_out/rowcost > $O/rowcost.log 2>&1 || { tail -5 $O/rowcost.log; exit 1; }
BG=nonzonal bash tools/gpu_sched_sweep.sh "" "--order total" "--first-chunk 24,160,300" "--first-chunk 24,96,240" "--chunk 480" || exit 1
for ord in priority cell; do
  timeout -k 10 400 python -u bench.py --config C5 --days 30 --steps 1 --warmup 1 --order $ord > $O/c5_$ord.log 2>&1 || { tail -5 $O/c5_$ord.log; exit 1; }
  grep '^{' $O/c5_$ord.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 $ord', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'])"
done
