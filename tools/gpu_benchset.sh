#!/bin/bash
# Bench lines of every config on the current tree (one GPU box session).
# usage: tools/gpu_benchset.sh <tag>
set -e
O=gpurun_out/benchset_$1; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/c3.json 2> $O/c3.err
for c in c1 c2 c2nm c3deep c5; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu --concurrency 0 > $O/$c.json 2> $O/$c.err
done
timeout -k 10 600 python -u bench.py --config c4 --steps 20 --no-cpu --concurrency 0 > $O/c4.json 2> $O/c4.err
timeout -k 10 600 python -u bench.py --config c4l0 --steps 20 --no-cpu --concurrency 0 > $O/c4l0.json 2> $O/c4l0.err
echo done > $O/done.txt
