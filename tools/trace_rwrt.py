"""Timeline of the rwrt kernels in a rocprofv3 --kernel-trace CSV: the last
`--last` dispatches (start relative to the first rwrt dispatch, duration).

    python tools/trace_rwrt.py <trace dir> [--last N]
"""
import csv
import glob
import sys

last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 40
rows = []
for p in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    with open(p) as fh:
        for r in csv.DictReader(fh):
            if "rwrt::" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
t0 = rows[0][0]
for s, e, n in rows[-last:]:
    print(f"{(s - t0) / 1e6:10.3f} ms {(e - s) / 1e6:9.3f} ms  {n.split('(')[0].replace('void ', '')[:60]}")
