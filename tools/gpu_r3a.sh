#!/bin/bash
# Round 3, first GPU pass: the GPU suite and smoke on the round-2 tree, and the
# per-ray 90-day C3 costs that pick the 90-day parity sample.
set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 300 python -u tools/c3_cost90.py --out gpurun_out/r3a > gpurun_out/r3a/cost90.log 2>&1 || { tail -20 gpurun_out/r3a/cost90.log; exit 1; }
cat gpurun_out/r3a/cost90.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3a/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3a/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3a/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3a/smoke.log 2>&1 || { tail gpurun_out/r3a/smoke.log; exit 1; }
tail -1 gpurun_out/r3a/smoke.log
