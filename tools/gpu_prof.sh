#!/bin/bash
# Profile the match kernels on the GPU box: timing, kernel trace, PMC passes.
# usage: tools/gpu_prof.sh <tag> [profile_walk.py args...]
set -e
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/profile_walk.py "$@" > $OUT/timing.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python -u tools/profile_walk.py "$@" > $OUT/trace.log 2>&1
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $pmc -d $OUT/pmc$i -o run --output-format csv -- python -u tools/profile_walk.py "$@" > $OUT/pmc$i.log 2>&1 || echo "pmc pass $i ($pmc) failed" >> $OUT/errors.txt
done
