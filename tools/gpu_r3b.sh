#!/bin/bash
# Round 3, pass B: the new horizon tests (C3 90 d, C5 10 d / 41 levels), the
# whole GPU suite on the rebuilt library, the weak-scaling bench (1 GPU and a
# 2-rank one-GPU rehearsal started by bench.py itself), a short C5 line.
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
grep -E "passed|failed" $O/pytest_gpu.log | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_n1.log 2>&1 || { tail -20 $O/bench_n1.log; exit 1; }
grep '^{' $O/bench_n1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N1', d['value'], d['ms_per_step'], d['scaling'], d['endpoints_rank0_sha256'], d['roofline']['frac'], d.get('bitwise_vs_cpu_oracle',{}).get('identical_values_frac'))"
timeout -k 10 600 python -u bench.py --gpus 2 --days 30 --steps 2 --warmup 1 > $O/bench_n2_shared.log 2>&1 || { tail -20 $O/bench_n2_shared.log; exit 1; }
grep '^{' $O/bench_n2_shared.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N2', d['n_gpus'], d['value'], d['scaling'], d['endpoints_rank0_sha256'], d.get('gathered_endpoints'))"
timeout -k 10 600 python -u bench.py --days 30 --steps 2 --warmup 1 --no-cpu > $O/bench_n1_30d.log 2>&1 || { tail -20 $O/bench_n1_30d.log; exit 1; }
grep '^{' $O/bench_n1_30d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N1-30d', d['value'], d['endpoints_rank0_sha256'])"
timeout -k 10 600 python -u bench.py --config C5 --days 10 --steps 1 --warmup 1 > $O/bench_c5_10d.log 2>&1 || { tail -20 $O/bench_c5_10d.log; exit 1; }
grep '^{' $O/bench_c5_10d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', d['value'], d['parity_sample_vs_oracle'])"
