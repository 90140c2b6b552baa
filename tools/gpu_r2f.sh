#!/bin/bash
# round 2 session f: GPU suite on the product library, variant timing, C3deep and C2 bench lines
mkdir -p gpurun_out/r2f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2f/gputest.log 2>&1; tail -3 gpurun_out/r2f/gputest.log
NOTEST=1 bash tools/gpu_variants.sh r2f --batches 20
cat gpurun_out/var_r2f/timing.txt
timeout -k 10 300 python -u bench.py --config c3deep --steps 20 > gpurun_out/r2f/c3deep.json 2> gpurun_out/r2f/c3deep.err; cat gpurun_out/r2f/c3deep.json
timeout -k 10 300 python -u bench.py --config c2 --steps 20 --no-cpu > gpurun_out/r2f/c2.json 2> gpurun_out/r2f/c2.err; cat gpurun_out/r2f/c2.json
