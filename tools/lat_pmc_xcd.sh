# The latency mode's per-attempt cycles grow with the number of XCDs that run
# latency blocks (profiles/r4/sched/latency_xcd.txt): PMC of the heaviest C3
# rays alone at 4 rays per wave on 4 vs 8 vs 16 CUs (one CU per XCD up to 8).
#   bash tools/lat_pmc_xcd.sh   (GPU box; each pass under its own time limit)
set -e
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 120 python3 tools/latency_only.py --find $O/heavy.npy
for k in 64 128 256; do
  timeout -k 10 60 python3 tools/latency_only.py --load $O/heavy.npy --k $k --density 4
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQC_ICACHE_MISSES SQC_DCACHE_MISSES SQ_INSTS_SMEM SQ_INSTS_VALU --kernel-trace -d $O/a$k -o run --output-format csv -- python3 tools/latency_only.py --load $O/heavy.npy --k $k --density 4 > $O/a$k.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQC_TC_INST_REQ SQC_TC_DATA_READ_REQ SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-trace -d $O/b$k -o run --output-format csv -- python3 tools/latency_only.py --load $O/heavy.npy --k $k --density 4 > $O/b$k.log 2>&1
done
python3 - <<'PY'
import csv, glob
for k in (64, 128, 256):
    c = {}
    for f in glob.glob(f"gpurun_out/r4u/[ab]{k}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rk45_run_kernel" in r["Kernel_Name"]:
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    w = c.get("SQ_WAVE_CYCLES", 1.0)
    print(k, {n: (round(v / w, 4) if n.startswith("SQ_WAIT") else v) for n, v in sorted(c.items())})
PY
for k in 64 128 256; do rm -rf $O/a$k $O/b$k; done
