#!/bin/bash
# Round-3 tree: bench lines of every config, then the N=2 bench rehearsal on
# one GPU (two ranks over gloo, as the driver launches N > 1 with torchrun).
# usage: tools/gpu_r3_benchset.sh <tag>
set -e
bash tools/gpu_benchset.sh $1
O=gpurun_out/benchset_$1
TM_BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 30 --warmup 3 --no-cpu --concurrency 0 \
  > $O/n2_rehearsal.json 2> $O/n2_rehearsal.err
