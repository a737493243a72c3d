"""Per-launch HBM traffic of rk45_run_kernel from two rocprofv3 PMC passes.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <bench_json_log> <out.json>

FETCH_SIZE and WRITE_SIZE (KiB, from the L2's memory-side request counters)
are collected in separate passes (TCC slots).  Following MI355X_MICROARCH.md
§HBM, FETCH_SIZE is doubled on gfx950 (it tallies 128-B requests at 64 B for
wide reads; our reads are a mix of 16-B gathers and streams -- uncalibrated,
so the doubled figure is an upper estimate of the read side).
"""
import csv
import json
import sys


def per_launch(d, counter):
    vals = []
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if "rk45_run_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    fetch_dir, write_dir, log, out = sys.argv[1:5]
    f = per_launch(fetch_dir, "FETCH_SIZE")
    w = per_launch(write_dir, "WRITE_SIZE")
    bench = None
    for line in open(log):
        if line.startswith("{"):
            bench = json.loads(line)
    n = min(len(f), len(w))
    fb, wb = sum(f[:n]) / n, sum(w[:n]) / n
    steps_per_launch = bench["ray_steps_per_step"] / (bench["roofline"]["launches"] / bench["steps"])
    res = {"workload": bench["config"]["workload"], "launch_rows": bench["config"].get("launch_rows"),
           "kernel": "rk45_run_kernel", "launches": n,
           "fetch_bytes_per_launch_x2": 2 * fb, "write_bytes_per_launch": wb,
           "traffic_bytes_per_launch": 2 * fb + wb,
           "algorithmic_bytes_per_launch": steps_per_launch * bench["roofline"]["bytes_per_ray_step"],
           "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE; counters in KiB x 1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
