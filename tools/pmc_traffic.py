"""Per-launch HBM traffic of one rwrt_rk45_run call (rk45_run_kernel plus the
frozen-ray flag and fill kernels it launches beside it) from two rocprofv3 PMC
passes.

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


KERNELS = ("rk45_run_kernel", "frozen_fill_kernel", "frozen_flag_kernel", "frozen_tail_kernel")


def per_launch(d, counter):
    """Bytes per rwrt_rk45_run call: the calls' kernels summed, divided over
    the rk45_run_kernel dispatches (one per call)."""
    total, launches = 0.0, 0
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] == counter and any(k in r["Kernel_Name"] for k in KERNELS):
            total += float(r["Counter_Value"]) * 1024.0
            launches += "rk45_run_kernel" in r["Kernel_Name"]
    return [total / max(launches, 1)] * launches


def by_kernel(d, counter):
    """Bytes per call of each of the call's kernels (run kernel dispatches = calls)."""
    tot, launches = {}, 0
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
        if k:
            tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0
            launches += k == "rk45_run_kernel"
    return {k: v / max(launches, 1) for k, v in tot.items()}


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
    launches_per_step = len(bench["config"]["launch_rows"])
    steps_per_launch = bench["ray_steps_per_step"] / launches_per_step
    bps = bench["roofline"].get("bytes_per_ray_step") or bench["roofline"]["algorithmic"]["bytes_per_ray_step"]
    res = {"workload": bench["config"]["workload"], "launch_rows": bench["config"].get("launch_rows"),
           "library_sha256": bench.get("library_sha256"),
           "kernel": "rk45_run_kernel", "kernels_summed": list(KERNELS), "launches": n,
           "fetch_bytes_per_launch_x2": 2 * fb, "write_bytes_per_launch": wb,
           "traffic_bytes_per_launch": 2 * fb + wb,
           "write_bytes_per_launch_by_kernel": by_kernel(write_dir, "WRITE_SIZE"),
           "fetch_bytes_per_launch_by_kernel_x2": {k: 2 * v for k, v in by_kernel(fetch_dir, "FETCH_SIZE").items()},
           "algorithmic_bytes_per_launch": steps_per_launch * bps,
           "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE; counters in KiB x 1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
