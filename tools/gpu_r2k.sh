#!/bin/bash
# emit variants: parity subset + C2 timing; bulk deltas (run patches) on the product library
mkdir -p gpurun_out/r2k
timeout -k 10 400 python -u tools/bulk_deltas.py > gpurun_out/r2k/bulk.json 2> gpurun_out/r2k/bulk.err; cat gpurun_out/r2k/bulk.json
bash tools/gpu_variants.sh r2k_c2 --config c2 --batches 12
cat gpurun_out/var_r2k_c2/timing.txt
