#!/bin/bash
# Round-2: C4 rehearsal on one GPU, N=2 rehearsal of the multi-rank bench path
# (gloo, ranks sharing the GPU), the host CPU's VRCP14PD table.
set -o pipefail
mkdir -p gpurun_out
gcc -O2 -mavx512f tools/rcp14_probe.c -o /tmp/rcp14_probe && /tmp/rcp14_probe gpurun_out/rcp14_box.bin && sha256sum gpurun_out/rcp14_box.bin
timeout -k 10 300 python tools/c4_rehearsal.py --out gpurun_out/c4_rehearsal.json > gpurun_out/c4_rehearsal.log 2>&1 || exit 1
RWRT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu \
  > gpurun_out/n2_gloo.log 2>&1 || exit 1
grep -h '^{' gpurun_out/n2_gloo.log | tail -c 1500
