#!/bin/bash
# Kernel trace + PMC passes over the walk driver for several library builds
# (TM_LIB): one rocprofv3 run per (library, pass).  PASSES holds the counter
# groups, ';'-separated; "trace" is the kernel trace.
# usage: PASSES="trace;SQ_WAVES SQ_INSTS_VALU" tools/gpu_libs_prof.sh <tag> <lib.so>... -- [profile_walk.py args]
set -e
TAG=$1; shift
OUT=gpurun_out/libs_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" = "--" ] && shift
IFS=';' read -ra passes <<< "${PASSES:-trace}"
for so in "${libs[@]}"; do
  name=$(basename $so .so)
  i=0
  for pmc in "${passes[@]}"; do
    i=$((i+1))
    if [ "$pmc" = "trace" ]; then
      TM_LIB=$so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$name/p$i -o run --output-format csv -- \
        python3 -u tools/profile_walk.py "$@" > $OUT/$name.p$i.log 2>&1
    else
      TM_LIB=$so timeout -k 10 -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/$name/p$i -o run --output-format csv -- \
        python3 -u tools/profile_walk.py "$@" > $OUT/$name.p$i.log 2>&1
    fi
  done
done
echo done > $OUT/done.txt
