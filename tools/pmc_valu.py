"""VALU issue of the ray-loop kernel from one rocprofv3 PMC pass.

    python tools/pmc_valu.py <pmc_dir> <bench_json_log> <out.json>

The pass collects SQ_INSTS_VALU (vector wave-instructions issued), SQ_WAVES,
SQ_WAVE_CYCLES, SQ_ACTIVE_INST_VALU, SQ_ACTIVE_INST_ANY and GRBM_GUI_ACTIVE.
rk45_run_kernel runs one wave per SIMD (1024 waves on 256 CUs x 4 SIMDs); a
VALU wave-instruction of one wave alone holds its SIMD's issue for at least 4
cycles (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'; fp64 FMA is
4 cycles per wave64 at the 16-lane fp64 rate).  The in-kernel clock is
GRBM_GUI_ACTIVE / 8 (XCDs) / kernel time (MI355X_MICROARCH.md 'DVFS
give-back').  Issue fraction = SQ_INSTS_VALU x 4 / (1024 x clock x time).
"""
import csv
import json
import sys

KERNEL = "rk45_run_kernel"


def main():
    d, log, out = sys.argv[1:4]
    per = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if KERNEL not in r["Kernel_Name"]:
            continue
        k = r["Dispatch_Id"]
        e = per.setdefault(k, {"t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    bench = None
    for line in open(log):
        if line.startswith("{"):
            bench = json.loads(line)
    launches = list(per.values())
    n = len(launches)
    tot = lambda c: sum(x.get(c, 0.0) for x in launches)
    t = tot("t")
    clock = tot("GRBM_GUI_ACTIVE") / 8.0 / t
    insts = tot("SQ_INSTS_VALU") / n
    res = {"workload": bench["config"]["workload"], "launch_rows": bench["config"].get("launch_rows"),
           "library_sha256": bench.get("library_sha256"),
           "kernel": KERNEL, "launches": n, "valu_insts_per_launch": insts,
           "clock_hz": clock, "simds": 1024, "cycles_per_valu": 4,
           "profiled_launch_ms": 1e3 * t / n,
           "frac_profiled": insts * 4 / (1024 * clock * t / n),
           "valu_active_frac": tot("SQ_ACTIVE_INST_VALU") / max(tot("SQ_WAVE_CYCLES"), 1.0),
           "issue_active_frac": tot("SQ_ACTIVE_INST_ANY") / max(tot("SQ_WAVE_CYCLES"), 1.0),
           "waves_per_launch": tot("SQ_WAVES") / n,
           "note": "SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE/8/time x time)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
