#!/bin/bash
# GPU parity on the product library, variant timing, C3deep bench line
mkdir -p gpurun_out/r2g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2g/gputest.log 2>&1; tail -3 gpurun_out/r2g/gputest.log
NOTEST=1 bash tools/gpu_variants.sh r2g --batches 20
cat gpurun_out/var_r2g/timing.txt
timeout -k 10 300 python -u bench.py --config c3deep --steps 20 --no-cpu > gpurun_out/r2g/c3deep.json 2> gpurun_out/r2g/c3deep.err; cat gpurun_out/r2g/c3deep.json
