#!/bin/bash
# PMC passes over the walk driver for several library builds (TM_LIB), one
# rocprofv3 run per (library, counter group).
# usage: tools/gpu_pmc_libs.sh <tag> <lib.so>... -- [profile_walk.py args]
set -e
TAG=$1; shift
OUT=gpurun_out/pmcl_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" = "--" ] && shift
for so in "${libs[@]}"; do
  name=$(basename $so .so)
  i=0
  for pmc in "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
    i=$((i+1))
    TM_LIB=$so timeout -k 10 -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/$name/p$i -o run --output-format csv -- \
      python3 -u tools/profile_walk.py "$@" > $OUT/$name.p$i.log 2>&1
  done
done
echo done > $OUT/done.txt
