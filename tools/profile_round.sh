#!/bin/bash
# Round profile on the GPU box: kernel-trace stats + FETCH/WRITE/SQ PMC passes
# of the bench command.  Raw output and summaries go to gpurun_out/prof_<round>/
# (merged back by gpurun); copy the summary/ directory into profiles/<round>/.
#   tools/profile_round.sh r1 [bench args]
set -e
r=$1; shift
export TMPDIR=/tmp
out=gpurun_out/prof_$r; sum=$out/summary; mkdir -p $out $sum
B="python3 bench.py --steps 2 --warmup 1 --no-cpu $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- $B > $out/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch -o run --output-format csv -- $B > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/write -o run --output-format csv -- $B > $out/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d $out/valu -o run --output-format csv -- $B > $out/valu.log 2>&1
# L2 hit rate and L2 -> fabric reads of the ray loop (3 of the 4 TCC slots)
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace -d $out/tcc -o run --output-format csv -- $B > $out/tcc.log 2>&1 || echo "tcc pass failed (see tcc.log)"
cp $out/trace/run_kernel_stats.csv $sum/kernel_stats.csv
python3 tools/pmc_traffic.py $out/fetch $out/write $out/trace.log $sum/traffic.json
python3 tools/pmc_valu.py $out/valu $out/trace.log $sum/valu.json
python3 tools/pmc_tcc.py $out/tcc $sum/tcc.json || true
# the run kernel's rows only (the whole collection of a C5 line is ~20 MB)
python3 -c "import sys; L=open(sys.argv[1]).read().splitlines(); open(sys.argv[2],'w').write('\\n'.join([L[0]]+[l for l in L[1:] if 'rk45_run_kernel' in l])+'\\n')" \
  $out/valu/run_counter_collection.csv $sum/valu_counters.csv
grep -h '^{' $out/trace.log > $sum/bench_under_rocprof.json || true
# keep the summaries only (the raw per-dispatch CSVs of a long run exceed
# gpurun's 64 MiB merge-back limit)
rm -rf $out/trace $out/fetch $out/write $out/valu $out/tcc
