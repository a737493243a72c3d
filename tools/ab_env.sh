#!/bin/bash
# Interleaved A/B bench lines of (environment, library) variants on one box.
#   tools/ab_env.sh <reps> "<bench args>" "<ENV=.. ENV=..>|<lib or ->" ...
# Prints one summary line per run: variant, value, ms/step, avg launch ms, endpoint hash.
set -o pipefail
reps=$1; args=$2; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 $reps); do
  i=0
  for spec in "$@"; do
    i=$((i + 1))
    envs=${spec%%|*}; lib=${spec#*|}
    L=(); [ "$lib" != "-" ] && L=(--lib $lib)
    f=gpurun_out/ab/v${i}_r$r.log
    env $envs timeout -k 10 600 python -u bench.py --no-cpu $args "${L[@]}" > $f 2>&1 || { tail -20 $f; exit 1; }
    grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$r', '$spec', '%.4g' % d['value'], '%.2f' % d['ms_per_step'], '%.2f' % r['avg_launch_ms'], d.get('endpoints_rank0_sha256'))"
  done
done
