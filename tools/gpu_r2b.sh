#!/bin/bash
# Round-2 GPU session b: multi-rank drop-in test, C5 at BASELINE size (fp64/fp32), C3 non-zonal line.
set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "world2 or multirank" > gpurun_out/r2b/pytest_multirank.log 2>&1 || { tail -30 gpurun_out/r2b/pytest_multirank.log; exit 1; }
tail -2 gpurun_out/r2b/pytest_multirank.log
timeout -k 10 400 python bench.py --config C5 --steps 1 --warmup 1 > gpurun_out/r2b/c5_fp64.log 2>&1 || { tail -20 gpurun_out/r2b/c5_fp64.log; exit 1; }
grep '^{' gpurun_out/r2b/c5_fp64.log | cut -c1-700
timeout -k 10 400 python bench.py --config C5 --fields fp32 --steps 1 --warmup 1 > gpurun_out/r2b/c5_fp32.log 2>&1 || { tail -20 gpurun_out/r2b/c5_fp32.log; exit 1; }
grep '^{' gpurun_out/r2b/c5_fp32.log | cut -c1-700
timeout -k 10 300 python bench.py --bg nonzonal --steps 3 --warmup 1 --no-cpu > gpurun_out/r2b/c3_nonzonal.log 2>&1 || { tail -20 gpurun_out/r2b/c3_nonzonal.log; exit 1; }
grep '^{' gpurun_out/r2b/c3_nonzonal.log | cut -c1-400
