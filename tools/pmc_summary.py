"""Summarise rocprofv3 SQ counter CSVs for rk45_run_kernel: python tools/pmc_summary.py <dir>..."""
import collections
import csv
import glob
import json
import sys


def load(d):
    out = collections.defaultdict(float)
    n = 0
    for f in glob.glob(f"{d}/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "rk45_run_kernel" in r["Kernel_Name"]:
                out[r["Counter_Name"]] += float(r["Counter_Value"])
                n += 1
    return out


def main():
    for tag in sys.argv[1:]:
        c = load(f"gpurun_out/pmc_{tag}_a")
        c.update(load(f"gpurun_out/pmc_{tag}_b"))
        wc = c["SQ_WAVE_CYCLES"] or 1
        summ = {k: round(c[k] / wc, 3) for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS")}
        summ["lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / max(c["SQ_ACTIVE_INST_VALU"] * 64, 1), 3)
        summ["valu_insts"] = c["SQ_INSTS_VALU"]
        summ["lds_insts"] = c["SQ_INSTS_LDS"]
        summ["vmem_rd"] = c["SQ_INSTS_VMEM_RD"]
        summ["salu"] = c["SQ_INSTS_SALU"]
        summ["smem"] = c["SQ_INSTS_SMEM"]
        print(tag, json.dumps(summ))


if __name__ == "__main__":
    main()
