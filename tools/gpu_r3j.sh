#!/bin/bash
# pass J: sliced work queue -- parity (edge cases, C3 90 d sliced), the GPU
# suite, bench A/B (unsliced vs sliced), tail traces.
set -o pipefail
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge_cases.py -x -v --timeout 120 --timeout-method thread > $O/pytest_edge.log 2>&1 || { tail -30 $O/pytest_edge.log; exit 1; }
grep -E "passed|failed" $O/pytest_edge.log | tail -1
timeout -k 10 400 python -u -m pytest tests/test_gpu_c3_ref90.py -x -v -k sliced --timeout 200 --timeout-method thread > $O/pytest_sliced90.log 2>&1 || { tail -30 $O/pytest_sliced90.log; exit 1; }
grep -E "passed|failed" $O/pytest_sliced90.log | tail -1
for args in "--bg zonal" "--bg zonal --slice 30" "--bg nonzonal" "--bg nonzonal --slice 30" "--bg nonzonal --slice 10"; do
  timeout -k 10 300 python -u bench.py --no-cpu $args > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $args', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'], d['endpoints_rank0_sha256'])"
done
timeout -k 10 300 python -u tools/tail_trace.py --bg nonzonal zonal --out $O > $O/tail0.log 2>&1 || { tail -5 $O/tail0.log; exit 1; }
cat $O/tail0.log
timeout -k 10 300 python -u tools/tail_trace.py --bg nonzonal zonal --slice 30 --out $O > $O/tail30.log 2>&1 || { tail -5 $O/tail30.log; exit 1; }
cat $O/tail30.log
