#!/bin/bash
# GPU parity, C3deep bench, C2 emit profile (kernel trace + PMC)
mkdir -p gpurun_out/r2i
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2i/gputest.log 2>&1; tail -3 gpurun_out/r2i/gputest.log
timeout -k 10 300 python -u bench.py --config c3deep --steps 20 --no-cpu > gpurun_out/r2i/c3deep.json 2> gpurun_out/r2i/c3deep.err; cut -c1-900 gpurun_out/r2i/c3deep.json
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2i/c2trace -o run --output-format csv -- python3 -u tools/profile_walk.py --config c2 --batches 8 > gpurun_out/r2i/c2trace.log 2>&1
for pmc in "WRITE_SIZE" "FETCH_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $pmc -d gpurun_out/r2i/c2pmc$i -o run --output-format csv -- python3 -u tools/profile_walk.py --config c2 --batches 8 > gpurun_out/r2i/c2pmc$i.log 2>&1
done
cat gpurun_out/r2i/c2trace/run_kernel_stats.csv
