#!/bin/bash
# Round 3, pass C: the shared-reciprocal division build -- device exactness
# test first, then the whole GPU suite, then the bench (C3 zonal, non-zonal).
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "math_exactness or t0 or t1" > $O/pytest_exact.log 2>&1 || { tail -30 $O/pytest_exact.log; exit 1; }
grep -E "passed|failed" $O/pytest_exact.log | tail -1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
grep -E "passed|failed" $O/pytest_gpu.log | tail -1
timeout -k 10 600 python -u bench.py --no-cpu > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['endpoints_rank0_sha256'], d['library_sha256'])"
timeout -k 10 600 python -u bench.py --no-cpu --bg nonzonal > $O/bench_nz.log 2>&1 || { tail -20 $O/bench_nz.log; exit 1; }
grep '^{' $O/bench_nz.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench-nz', d['value'], d['ms_per_step'], d['endpoints_rank0_sha256'])"
