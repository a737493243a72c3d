#!/bin/bash
# pass I: per-ray row costs (1/16 of the live rays, every 10th row) for the
# in-launch scheduling model; the latency trace with per-XCC clocks.
set -o pipefail
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 400 python -u tools/c3_row_costs.py --bg nonzonal zonal --skip-full --compact $O --sub 16 > $O/rowcost.log 2>&1 || { tail -5 $O/rowcost.log; exit 1; }
ls -la $O
timeout -k 10 600 python -u tools/latency_trace.py --out $O/latency_trace.json > $O/latency_trace.log 2>&1 || { tail -20 $O/latency_trace.log; exit 1; }
cat $O/latency_trace.log
