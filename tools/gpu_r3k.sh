#!/bin/bash
# pass K: A/B of the unsliced run kernel (HEAD build vs the sliced-queue build),
# latency-mode placement cases
set -o pipefail
O=gpurun_out/r3k
mkdir -p $O
for rep in 1 2; do
for lib in rossby-wave-ray-tracing_amd/librwrt_old.so rossby-wave-ray-tracing_amd/librwrt.so; do
  timeout -k 10 300 python -u bench.py --no-cpu --lib $lib > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
  grep '^{' $O/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('AB $lib', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['endpoints_rank0_sha256'])"
done
done
timeout -k 10 600 python -u tools/latency_trace.py --cases alone:4:1,alone:8:1,alone:64:16,alone:16:4,alone:1:1 --out $O/latency_trace2.json > $O/latency_trace2.log 2>&1 || { tail -20 $O/latency_trace2.log; exit 1; }
grep case $O/latency_trace2.log
