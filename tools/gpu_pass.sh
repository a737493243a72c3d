#!/bin/bash
# One GPU pass on the box, steps run in order, the first failure ends it
# (each step under its own time limit; logs under gpurun_out/<name>/).
#   tools/gpu_pass.sh <name> <step> [<step> ...]
# steps:
#   suite[:<pytest -k expr>]     the -m gpu suite (or the selected tests)
#   smoke                        __graft_entry__.smoke()
#   bench[:<bench.py args>]      one bench line (--no-cpu unless args say otherwise)
#   driver                       the driver's command: bench.py --gpus 1 (with the CPU baseline)
#   ab:<lib>,<lib>..:<reps>[:<bench args>]   interleaved A/B bench lines of library builds
#   prof:<tag>[:<bench args>]    same-build profile (tools/profile_round.sh <tag> <args>)
#   py:<script and args>         python3 <script and args>
#   sh:<command>                 any shell command (e.g. RWRT_LIB=... python3 tools/...)
set -o pipefail
name=$1; shift
O=gpurun_out/$name
mkdir -p $O
line() {   # summary of a bench JSON line on stdin
  python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print(d.get('value'), d.get('ms_per_step'), r.get('frac'), d.get('endpoints_rank0_sha256'), d.get('library'), d.get('library_sha256'))"
}
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  rest=${step#*:}
  [ "$rest" = "$step" ] && rest=""
  case $kind in
    suite)
      k=(); [ -n "$rest" ] && k=(-k "$rest")
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > $O/pytest_gpu_$n.log 2>&1 || { tail -40 $O/pytest_gpu_$n.log; exit 1; }
      grep -E "passed|failed" $O/pytest_gpu_$n.log | tail -1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 900 python -u bench.py --no-cpu $rest > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
      grep '^{' $O/bench_$n.log > $O/bench_$n.json
      echo "bench $rest: $(line < $O/bench_$n.json)" ;;
    driver)
      timeout -k 10 900 python -u bench.py --gpus 1 $rest > $O/bench_driver_$n.log 2>&1 || { tail -20 $O/bench_driver_$n.log; exit 1; }
      grep '^{' $O/bench_driver_$n.log > $O/bench_driver_$n.json
      echo "driver: $(line < $O/bench_driver_$n.json)" ;;
    ab)
      libs=${rest%%:*}; rest=${rest#*:}
      reps=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      for r in $(seq 1 $reps); do
        for lib in ${libs//,/ }; do
          f=$O/ab_${n}_$(basename $lib .so)_$r
          timeout -k 10 600 python -u bench.py --no-cpu --lib $lib $args > $f.log 2>&1 || { tail -20 $f.log; exit 1; }
          grep '^{' $f.log > $f.json
          echo "ab $r $(basename $lib): $(line < $f.json)"
        done
      done ;;
    prof)
      tag=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      bash tools/profile_round.sh $tag $args || exit 1
      S=gpurun_out/prof_$tag/summary
      timeout -k 10 900 python -u bench.py --no-cpu --valu-profile $S/valu.json --traffic $S/traffic.json $args \
        > $O/bench_prof_$tag.log 2>&1 || { tail -20 $O/bench_prof_$tag.log; exit 1; }
      grep '^{' $O/bench_prof_$tag.log > $S/bench_line.json
      echo "prof $tag: $(line < $S/bench_line.json)" ;;
    py)
      timeout -k 10 900 python3 -u $rest > $O/py_$n.log 2>&1 || { tail -30 $O/py_$n.log; exit 1; }
      tail -5 $O/py_$n.log ;;
    sh)
      timeout -k 10 900 bash -c "$rest" > $O/sh_$n.log 2>&1 || { tail -30 $O/sh_$n.log; exit 1; }
      tail -6 $O/sh_$n.log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
