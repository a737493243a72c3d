"""Summary of tools/pmc_stall.sh: the run kernel's SQ counters summed over its
dispatches, and the shares of wave cycles (per SIMD: one wave each).

    python tools/pmc_stall.py <dir with p1/ p2/ p3/>
"""
import csv
import glob
import json
import sys


def main():
    d = sys.argv[1]
    c = {}
    for f in glob.glob(f"{d}/p*/**/run_counter_collection.csv", recursive=True) + \
            glob.glob(f"{d}/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "rk45_run_kernel" in r["Kernel_Name"]:
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    wc = c.get("SQ_WAVE_CYCLES") or 1.0
    share = {k: c[k] / wc for k in c if k.startswith(("SQ_ACTIVE_INST", "SQ_WAIT", "SQ_INST_CYCLES", "SQ_BUSY"))}
    per_valu = {k: c[k] / max(c.get("SQ_INSTS_VALU", 1), 1) for k in c if k.startswith("SQ_INSTS")}
    lat = {"lds_cycles_per_inst": c.get("SQ_INST_LEVEL_LDS", 0) / max(c.get("SQ_INSTS_LDS", 1), 1),
           "vmem_rd_cycles_per_inst": c.get("SQ_INST_LEVEL_VMEM", 0) / max(c.get("SQ_INSTS_VMEM_RD", 1), 1)}
    out = {"counters": c, "share_of_wave_cycles": share, "per_valu_inst": per_valu, "latency": lat,
           "lane_util": c.get("SQ_THREAD_CYCLES_VALU", 0) / max(c.get("SQ_ACTIVE_INST_VALU", 1) * 64, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
