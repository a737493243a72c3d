set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/kt
for v in "r4:RWRT_TAILS=0:rossby-wave-ray-tracing_amd/librwrt_r4.so" "tails:RWRT_TAILS=1:rossby-wave-ray-tracing_amd/librwrt.so" "dense:RWRT_TAILS=0:rossby-wave-ray-tracing_amd/librwrt.so"; do
  n=${v%%:*}; r=${v#*:}; e=${r%%:*}; lib=${r#*:}
  export RWRT_TAILS=${e#RWRT_TAILS=}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/$n -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --lib $lib > gpurun_out/kt/$n.log 2>&1
  cp gpurun_out/kt/$n/run_kernel_stats.csv gpurun_out/kt/${n}_stats.csv
  rm -rf gpurun_out/kt/$n
done
