#!/bin/bash
# GPU check of the current tree: the -m gpu suite, smoke(), then a short bench
# (no CPU baseline).  Logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_nocpu.log 2>&1 || exit 1
grep -h '^{' gpurun_out/bench_nocpu.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
