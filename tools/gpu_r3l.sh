#!/bin/bash
# pass L: budgeted calls -- parity, A/B (classic path vs HEAD build; budgets on both backgrounds)
set -o pipefail
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge_cases.py -x -v --timeout 120 --timeout-method thread > $O/pytest_edge.log 2>&1 || { tail -30 $O/pytest_edge.log; exit 1; }
grep -E "passed|failed" $O/pytest_edge.log | tail -1
timeout -k 10 400 python -u -m pytest tests/test_gpu_c3_ref90.py -x -v -k budgeted --timeout 200 --timeout-method thread > $O/pytest_budget90.log 2>&1 || { tail -30 $O/pytest_budget90.log; exit 1; }
grep -E "passed|failed" $O/pytest_budget90.log | tail -1
b() {
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $*', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['config']['launch_rows'], d['endpoints_rank0_sha256'])"
}
b --lib rossby-wave-ray-tracing_amd/librwrt_old.so || exit 1
b || exit 1
b --budgets 60,60,60 --team 0 || exit 1
b --budgets 60,60,60 --team 128 || exit 1
b --budgets 40,40,40,40,40 --team 128 || exit 1
b --lib rossby-wave-ray-tracing_amd/librwrt_old.so || exit 1
b || exit 1
b --bg nonzonal || exit 1
b --bg nonzonal --budgets 60,60,60 --team 0 || exit 1
b --bg nonzonal --budgets 40,40,40,40,40 --team 0 || exit 1
timeout -k 10 300 python -u tools/tail_trace.py --bg nonzonal zonal --budgets 60,60,60 --team 0 --out $O > $O/tailb.log 2>&1 || { tail -5 $O/tailb.log; exit 1; }
cat $O/tailb.log
