#!/bin/bash
# Profile the match path on the GPU box: the bench command under a kernel
# trace (--stats), then one PMC pass per counter group over the minimal
# profiling driver.  Any failing / timed-out step ends the script (no retries).
# usage: tools/gpu_prof.sh <tag> [--no-bench] [profile_walk.py args...]
set -e
TAG=$1; shift
BENCH=1
if [ "$1" = "--no-bench" ]; then BENCH=0; shift; fi
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ $BENCH = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench -o run --output-format csv -- \
    python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
  # the bench's concurrent-caller leg launches ~10^5 kernels: keep the trace compressed
  gzip -f $OUT/bench/run_kernel_trace.csv
fi
timeout -k 10 200 python3 -u tools/profile_walk.py "$@" > $OUT/timing.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 -u tools/profile_walk.py "$@" > $OUT/trace.log 2>&1
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/pmc$i -o run --output-format csv -- \
    python3 -u tools/profile_walk.py "$@" > $OUT/pmc$i.log 2>&1
done
echo "profile $TAG done" > $OUT/done.txt
