#!/bin/bash
# Latency mode: parity tests, then its latency on the heaviest C3 rays.
set -o pipefail
mkdir -p gpurun_out/team
timeout -k 10 400 python -u -m pytest tests/test_gpu_team.py -x -v --timeout 300 --timeout-method thread > gpurun_out/team/pytest.log 2>&1 || { tail -30 gpurun_out/team/pytest.log; exit 1; }
tail -3 gpurun_out/team/pytest.log
timeout -k 10 300 python tools/team_latency.py --out gpurun_out/team/latency.json > gpurun_out/team/latency.log 2>&1 || { tail -20 gpurun_out/team/latency.log; exit 1; }
grep -v '"cases"' gpurun_out/team/latency.log
