#!/bin/bash
# Section cycles of the heaviest C3 ray alone (diagnostic stamps build).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamps.py "$@" > gpurun_out/stamps.json 2>gpurun_out/stamps.err || { tail gpurun_out/stamps.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/stamps.json"))
print(d["cycles_per_attempt"], d["refills_per_attempt"])
for k, v in d["sections"].items():
    print("%-45s %10.0f" % (k, v["cycles_per_attempt"]))
PY
timeout -k 10 200 python tools/stamps.py --batch --days 12 > gpurun_out/stamps_batch.json 2>>gpurun_out/stamps.err || { tail gpurun_out/stamps.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/stamps_batch.json"))
print("batch", d["cycles_per_attempt"], d["refills_per_attempt"])
for k, v in d["sections"].items():
    print("%-45s %6.3f" % (k, v["frac"]))
PY

