#!/bin/bash
# Study builds of libtmatch (emqx_amd/variants/libtmatch_<name>.so): walk timing
# on the profiling driver plus two PMC passes each.  A variant named
# "hostwids" runs with TM_STUDY_HOSTWIDS=1 (wids looked up on the host).
# usage: tools/gpu_study.sh <tag> <name>... -- [profile_walk.py args]
set -e
TAG=$1; shift
OUT=gpurun_out/study_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
names=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done
[ "$1" = "--" ] && shift
for v in "${names[@]}"; do
  so=emqx_amd/variants/libtmatch_$v.so
  if [ "$v" = hostwids ]; then export TM_STUDY_HOSTWIDS=1; else unset TM_STUDY_HOSTWIDS; fi
  echo "== $v" >> $OUT/timing.txt
  TM_LIB=$so timeout -k 10 150 python3 -u tools/profile_walk.py "$@" 2>&1 | grep -v amdgpu.ids >> $OUT/timing.txt
  i=0
  for pmc in "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    TM_LIB=$so timeout -k 10 -s KILL 150 rocprofv3 --pmc $pmc -d $OUT/$v/p$i -o run --output-format csv -- \
      python3 -u tools/profile_walk.py "$@" > $OUT/$v.p$i.log 2>&1
  done
done
echo done > $OUT/done.txt
