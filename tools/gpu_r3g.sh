#!/bin/bash
# pass G: cost of the (off) trace hook (A/B vs the qdiv build), then the latency trace
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
for rep in 1 2; do
for lib in rossby-wave-ray-tracing_amd/librwrt.so; do
  timeout -k 10 300 python -u bench.py --no-cpu --lib $lib > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
  grep '^{' $O/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('AB $lib', round(d['value']/1e9,4), round(d['ms_per_step'],1), d['endpoints_rank0_sha256'])"
done
done
timeout -k 10 600 python -u tools/latency_trace.py --out $O/latency_trace.json > $O/latency_trace.log 2>&1 || { tail -20 $O/latency_trace.log; exit 1; }
cat $O/latency_trace.log
