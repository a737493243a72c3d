#!/bin/bash
# Non-zonal C3 profile (stats + traffic + VALU) and an instruction-mix pass for both backgrounds.
set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh r2nz --bg nonzonal || exit 1
for bg in zonal nonzonal; do
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/mix_$bg -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --bg $bg > gpurun_out/mix_$bg.log 2>&1 || exit 1
done
echo ok
