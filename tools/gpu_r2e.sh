set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r2e.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_r2e.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_r2e.log | head -5
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh rossby-wave-ray-tracing_amd/librwrt.so rossby-wave-ray-tracing_amd/librwrt_chunkmajor.so || exit 1
bash tools/gpu_stamps.sh
