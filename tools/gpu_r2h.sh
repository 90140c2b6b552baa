#!/bin/bash
# GPU parity on the product library, C3deep and C3 bench lines
mkdir -p gpurun_out/r2h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2h/gputest.log 2>&1; tail -3 gpurun_out/r2h/gputest.log
timeout -k 10 300 python -u bench.py --config c3deep --steps 20 --no-cpu > gpurun_out/r2h/c3deep.json 2> gpurun_out/r2h/c3deep.err; cut -c1-1200 gpurun_out/r2h/c3deep.json
timeout -k 10 300 python -u bench.py > gpurun_out/r2h/c3.json 2> gpurun_out/r2h/c3.err; cut -c1-1500 gpurun_out/r2h/c3.json
