#!/bin/bash
# Interleaved A/B bench lines over bench.py argument sets on one box.
#   tools/ab_args.sh <reps> "<args A>" "<args B>" ...
# Prints one summary line per run: rep, args, value, ms/step, avg launch ms, endpoint hash.
set -o pipefail
reps=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 $reps); do
  i=0
  for args in "$@"; do
    i=$((i + 1))
    f=gpurun_out/ab/a${i}_r$r.log
    timeout -k 10 600 python -u bench.py --no-cpu $args > $f 2>&1 || { tail -20 $f; exit 1; }
    grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$r', '[$args]', '%.4g' % d['value'], '%.2f' % d['ms_per_step'], '%.2f' % r['avg_launch_ms'], d.get('endpoints_rank0_sha256'))"
  done
done
