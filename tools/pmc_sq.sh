#!/bin/bash
# SQ counter passes for one library variant: tools/pmc_sq.sh <tag> <lib> <days>
tag=$1; lib=$2; days=$3
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d gpurun_out/pmc_${tag}_a -o run --output-format csv -- python3 bench.py --days $days --steps 1 --warmup 0 --no-cpu --lib $lib > gpurun_out/pmc_${tag}_a.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM --kernel-trace -d gpurun_out/pmc_${tag}_b -o run --output-format csv -- python3 bench.py --days $days --steps 1 --warmup 0 --no-cpu --lib $lib > gpurun_out/pmc_${tag}_b.log 2>&1 || exit 1
