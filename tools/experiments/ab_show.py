"""Print one line per bench JSON line of an A/B log: value, library, config knobs."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        c = d["config"]
        print(f'{d["value"]:.4e} {d["ms_per_step"]:8.1f} ms  {d.get("library")} rows/launch={c.get("rows_per_launch")} '
              f'lead={c.get("launch_rows", [])[:-1][:6]} order={d.get("queue_order")} launches={d["roofline"]["launches"]} '
              f'avg={d["roofline"]["avg_launch_ms"]:.2f} ms')
