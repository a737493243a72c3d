#!/bin/bash
# PC sampling of the bench kernel: tools/pcsample.sh <tag> <method> <unit> <interval> [bench args]
tag=$1; method=$2; unit=$3; iv=$4; shift 4
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $method \
  --pc-sampling-unit $unit --pc-sampling-interval $iv -d gpurun_out/pcs_$tag -o pcs \
  --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" \
  > gpurun_out/pcs_$tag.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 gpurun_out/pcs_$tag.log; find gpurun_out/pcs_$tag -type f | head; exit $rc
