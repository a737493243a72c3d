#!/bin/bash
# Where the run kernel's wave cycles go: three SQ counter passes (at most 8 SQ
# counters each) of one bench command, summed over the rk45_run_kernel
# dispatches by tools/pmc_stall.py.   tools/pmc_stall.sh <tag> [bench args]
set -e
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/stall_$tag; mkdir -p $out
B="python3 bench.py --steps 1 --warmup 0 --no-cpu $*"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU"
P3="SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VMEM_TA_ADDR_FIFO_FULL SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F64"
P4="SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace -d $out/p$i -o run --output-format csv -- $B > $out/p$i.log 2>&1
done
python3 tools/pmc_stall.py $out > $out/summary.json
cat $out/summary.json
rm -rf $out/p1 $out/p2 $out/p3 $out/p4
