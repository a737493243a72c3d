#!/bin/bash
# Round 3, pass E: A/B of the cell-coordinate division (qdiv build vs current),
# the schedule model on the box (small output), more non-zonal schedules.
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
for rep in 1 2; do
for lib in rossby-wave-ray-tracing_amd/librwrt_qdiv.so rossby-wave-ray-tracing_amd/librwrt.so; do
  timeout -k 10 300 python -u bench.py --no-cpu --lib $lib > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
  grep '^{' $O/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('AB $lib', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['endpoints_rank0_sha256'])"
done
done
timeout -k 10 400 python -u tools/c3_row_costs.py --bg nonzonal zonal > $O/rowcost.log 2>&1 || { tail -5 $O/rowcost.log; exit 1; }
for k in nonzonal zonal; do timeout -k 10 300 python -u tools/sched_sim.py /tmp/rwrt_rowcost/c3_rowcost_$k.npz > $O/sim_$k.txt 2>&1 || { tail -5 $O/sim_$k.txt; exit 1; }; cat $O/sim_$k.txt; done
BG=nonzonal bash tools/gpu_sched_sweep.sh "--first-chunk 24,160,300 --order total" "--first-chunk 24,160,240,330" "--first-chunk 24,200,400" "--first-chunk 24,120,240,360" || exit 1
