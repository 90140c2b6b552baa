#!/bin/bash
# GPU suite; C3deep kernel trace and bench line
mkdir -p gpurun_out/r2m
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2m/gputest.log 2>&1; tail -3 gpurun_out/r2m/gputest.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2m/deeptrace -o run --output-format csv -- python3 -u tools/profile_walk.py --config c3deep --batches 8 > gpurun_out/r2m/deeptrace.log 2>&1
cut -c1-160 gpurun_out/r2m/deeptrace/run_kernel_stats.csv | head -6
timeout -k 10 300 python -u bench.py --config c3deep --steps 20 --no-cpu > gpurun_out/r2m/c3deep.json 2> gpurun_out/r2m/c3deep.err; cut -c1-400 gpurun_out/r2m/c3deep.json
