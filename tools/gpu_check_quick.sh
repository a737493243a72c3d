#!/bin/bash
# GPU suite + smoke + one bench line of the current tree (logs under gpurun_out/$1).
set -o pipefail
O=gpurun_out/${1:-check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
grep -E "passed|failed" $O/pytest_gpu.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py --no-cpu ${BENCH_ARGS} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['endpoints_rank0_sha256'], d['library_sha256'])"
