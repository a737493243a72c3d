set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "dropin or sink or great_circle" > gpurun_out/pytest_dropin.log 2>&1 || { tail -30 gpurun_out/pytest_dropin.log; exit 1; }
tail -3 gpurun_out/pytest_dropin.log
timeout -k 10 300 python tools/dropin_rate.py > gpurun_out/dropin_rate.json 2> gpurun_out/dropin_rate.err || { tail gpurun_out/dropin_rate.err; exit 1; }
cat gpurun_out/dropin_rate.json
