#!/bin/bash
# Profile summaries of the current build: C3 zonal and non-zonal bench schedules
# (rocprof kernel stats + FETCH/WRITE + SQ VALU passes; tools/profile_round.sh).
set -o pipefail
tag=${1:-r3}
bash tools/profile_round.sh ${tag}_zonal || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/prof_${tag}_zonal/summary/valu.json')); print('zonal', d['valu_insts_per_launch'], d['frac_profiled'], d['issue_active_frac'], d['valu_active_frac'], d['profiled_launch_ms'])"
bash tools/profile_round.sh ${tag}_nonzonal --bg nonzonal || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/prof_${tag}_nonzonal/summary/valu.json')); print('nonzonal', d['valu_insts_per_launch'], d['frac_profiled'], d['issue_active_frac'], d['valu_active_frac'], d['profiled_launch_ms'])"
