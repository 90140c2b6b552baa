#!/bin/bash
# GPU suite on the product library; C3deep kernel trace (where the deep topics' time goes)
mkdir -p gpurun_out/r2l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2l/gputest.log 2>&1; tail -3 gpurun_out/r2l/gputest.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2l/deeptrace -o run --output-format csv -- python3 -u tools/profile_walk.py --config c3deep --batches 8 > gpurun_out/r2l/deeptrace.log 2>&1
cut -c1-200 gpurun_out/r2l/deeptrace/run_kernel_stats.csv; cat gpurun_out/r2l/deeptrace.log | tail -2
