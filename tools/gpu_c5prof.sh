#!/bin/bash
# FETCH_SIZE calibration for the C5 gathers, then the C5 (BASELINE size) profile.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c5cal
hipcc --offload-arch=gfx950 -O3 -o /tmp/fetch_probe tools/probes/fetch_probe.hip || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/c5cal/probe -o run --output-format csv -- /tmp/fetch_probe > gpurun_out/c5cal/probe.log 2>&1 || exit 1
cat gpurun_out/c5cal/probe.log | grep requested
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/c5cal/probe/run_counter_collection.csv")):
    print(r["Kernel_Name"][:40], r["Counter_Name"], float(r["Counter_Value"]) * 1024)
PY
for f in fp64 fp32; do
  bash tools/profile_round.sh r2c5_$f --config C5 --fields $f || exit 1
done
