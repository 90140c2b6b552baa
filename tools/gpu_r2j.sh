#!/bin/bash
# emit variants: parity subset + C2 and C3 timing on the profiling driver
mkdir -p gpurun_out/r2j
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2j/gputest.log 2>&1; tail -3 gpurun_out/r2j/gputest.log
bash tools/gpu_variants.sh r2j_c2 --config c2 --batches 12
NOTEST=1 bash tools/gpu_variants.sh r2j_c3 --batches 12
cat gpurun_out/var_r2j_c2/timing.txt gpurun_out/var_r2j_c3/timing.txt
