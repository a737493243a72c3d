#!/bin/bash
# Instruction-cache hits/misses of the ray-loop kernel for library builds
# (code placement A/B): tools/icache_pmc.sh <lib> [<lib> ...]
export TMPDIR=/tmp
mkdir -p gpurun_out/icache
for lib in "$@"; do
  n=$(basename $lib .so)
  timeout -s KILL 180 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-trace -d gpurun_out/icache/$n -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --lib $lib > gpurun_out/icache/$n.log 2>&1 || { echo "$n: pmc pass failed"; tail -5 gpurun_out/icache/$n.log; continue; }
  python3 - gpurun_out/icache/$n/run_counter_collection.csv $n <<'PY'
import csv, sys
t = {}
for r in csv.DictReader(open(sys.argv[1])):
    if "rk45_run_kernel" in r["Kernel_Name"]:
        t[r["Counter_Name"]] = t.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
h, m = t.get("SQC_ICACHE_HITS", 0.0), t.get("SQC_ICACHE_MISSES", 0.0)
print(sys.argv[2], "icache hits %.4g misses %.4g miss rate %.5f" % (h, m, m / (h + m) if h + m else float("nan")))
PY
  rm -rf gpurun_out/icache/$n
done
