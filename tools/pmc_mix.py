"""Dynamic instruction mix of the ray-loop kernel from a rocprofv3 PMC pass
(SQ_INSTS, SQ_INSTS_VALU / _SALU / _LDS / _SMEM / _BRANCH, SQ_WAIT_INST_ANY,
SQ_WAVES), summed over the rk45_run_kernel dispatches of the run; with a
second pass (SQC_ICACHE_HITS / _MISSES) if given.

    python tools/pmc_mix.py <pmc_dir> [<sqc_dir>]
"""
import csv
import json
import sys


def sums(d, kernel="rk45_run_kernel"):
    tot = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if kernel in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return tot


t = sums(sys.argv[1])
out = {"counters": t}
if t.get("SQ_INSTS"):
    out["share_of_issued"] = {k: t[k] / t["SQ_INSTS"] for k in t if k.startswith("SQ_INSTS_")}
    out["salu_per_valu"] = t.get("SQ_INSTS_SALU", 0) / max(t.get("SQ_INSTS_VALU", 1), 1)
if len(sys.argv) > 2:
    q = sums(sys.argv[2])
    out["sqc"] = q
    h, m = q.get("SQC_ICACHE_HITS", 0), q.get("SQC_ICACHE_MISSES", 0)
    if h + m:
        out["icache_miss_rate"] = m / (h + m)
print(json.dumps(out, indent=1))
