set -o pipefail
mkdir -p gpurun_out/sweep
CFGS=${SWEEP:-"6:24,96 6:24,128"}
for c in $CFGS; do cfg=${c/:/ }
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --probe $1 --first-chunk $2 > gpurun_out/sweep/p$1_$2.log 2>&1 || { tail -3 gpurun_out/sweep/p$1_$2.log; exit 1; }
  grep -h '^{' gpurun_out/sweep/p$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('probe $1 lead $2', round(d['value']/1e9,4), round(d['ms_per_step'],2))"
done
