#!/bin/bash
# Round-4 tree: bench lines of the other configs (part a: c1 c2 c2nm c3deep c5 and the
# N=2 rehearsal over gloo on one GPU; part b: the 100M-filter c4 / c4l0 lines).
# usage: tools/gpu_r4_benchset.sh <tag> a|b
set -e
O=gpurun_out/benchset_$1; mkdir -p $O
if [ "$2" = a ]; then
  for c in c1 c2 c2nm c3deep c5; do
    timeout -k 10 400 python -u bench.py --config $c --no-cpu --concurrency 0 > $O/$c.json 2> $O/$c.err
  done
  TM_BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 30 --warmup 3 --no-cpu --concurrency 0 \
    > $O/n2_rehearsal.json 2> $O/n2_rehearsal.err
else
  timeout -k 10 600 python -u bench.py --config c4 --steps 20 --no-cpu --concurrency 0 > $O/c4.json 2> $O/c4.err
  timeout -k 10 600 python -u bench.py --config c4l0 --steps 20 --no-cpu --concurrency 0 > $O/c4l0.json 2> $O/c4l0.err
fi
echo done > $O/done_$2.txt
