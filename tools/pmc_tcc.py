"""L2 (TCC) hit rate of the ray-loop kernel from a rocprofv3 PMC pass
(TCC_HIT_sum, TCC_MISS_sum, TCC_EA0_RDREQ_sum; MI355X_MICROARCH.md §L2).

    python tools/pmc_tcc.py <tcc_dir> <out.json>

Per rk45_run_kernel dispatch: hits, misses, hit rate, and the L2's read
requests to the fabric (served by the Infinity Cache or HBM; x 64 B is
FETCH_SIZE)."""
import csv
import json
import sys


def main():
    d, out = sys.argv[1:3]
    tot, n = {}, 0
    seen = set()
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if "rk45_run_kernel" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        seen.add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    n = max(len(seen), 1)
    hit, miss, rd = (tot.get(k, 0.0) / n for k in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum"))
    res = {"kernel": "rk45_run_kernel", "dispatches": len(seen), "tcc_hit_per_launch": hit,
           "tcc_miss_per_launch": miss, "tcc_hit_rate": hit / (hit + miss) if hit + miss else None,
           "tcc_ea0_rdreq_per_launch": rd, "fabric_read_bytes_per_launch_x64": 64.0 * rd,
           "note": "TCC_EA0_RDREQ counts the L2's read requests to the fabric (Infinity Cache hits included)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
