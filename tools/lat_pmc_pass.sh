set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r4k
python3 tools/latency_only.py --find gpurun_out/r4k/heavy.npy
for d in 4 16; do
  python3 tools/latency_only.py --load gpurun_out/r4k/heavy.npy --k 256 --density $d
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_IFETCH SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/r4k/d$d -o run --output-format csv -- python3 tools/latency_only.py --load gpurun_out/r4k/heavy.npy --k 256 --density $d > gpurun_out/r4k/d$d.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/r4k/e$d -o run --output-format csv -- python3 tools/latency_only.py --load gpurun_out/r4k/heavy.npy --k 256 --density $d > gpurun_out/r4k/e$d.log 2>&1
done
python3 - <<'PY'
import csv, glob
for d in (4, 16):
    c = {}
    for f in glob.glob(f"gpurun_out/r4k/[de]{d}/**/run_counter_collection.csv", recursive=True) + glob.glob(f"gpurun_out/r4k/[de]{d}/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "rk45_run_kernel" in r["Kernel_Name"]:
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print(d, {k: (round(v / c["SQ_WAVE_CYCLES"], 4) if k.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY", "SQ_INST_CYCLES")) else v) for k, v in sorted(c.items())})
PY
rm -rf gpurun_out/r4k/d4 gpurun_out/r4k/d16 gpurun_out/r4k/e4 gpurun_out/r4k/e16
