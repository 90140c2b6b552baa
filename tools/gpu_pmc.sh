#!/bin/bash
# Extra PMC passes over the profiling driver, one rocprofv3 run per group.
# usage: tools/gpu_pmc.sh <tag> "<counters pass 1>" ["<counters pass 2>" ...] -- [profile_walk.py args]
set -e
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
passes=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do passes+=("$1"); shift; done
[ "$1" = "--" ] && shift
i=0
for pmc in "${passes[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/p$i -o run --output-format csv -- \
    python3 -u tools/profile_walk.py "$@" > $OUT/p$i.log 2>&1
done
echo done > $OUT/done.txt
