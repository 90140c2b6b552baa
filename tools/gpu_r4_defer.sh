#!/bin/bash
# Round 4: k_walk_one parking study -- the new GPU tests (unless NOTESTS=1), then
# the walk driver per build (product + emqx_amd/variants) x LB_DEFER x streams,
# and the two-phase path for reference.
# usage: tools/gpu_r4_defer.sh <tag> [profile_walk.py args]
set -e
TAG=$1; shift
OUT=gpurun_out/var_$TAG
mkdir -p $OUT
if [ -z "$NOTESTS" ]; then
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "one_pass or lookback or parked or u32 or boot_1m" > $OUT/tests.log 2>&1 || {
  rc=$?; echo "tests rc=$rc" >> $OUT/timing.txt; [ $rc -eq 1 ] || exit $rc; }
fi
for st in 1 3; do
  echo "== product phases streams=$st" >> $OUT/timing.txt
  timeout -k 10 120 python3 -u tools/profile_walk.py --large-path phases --streams $st "$@" 2>&1 | grep -v amdgpu.ids >> $OUT/timing.txt
done
for so in emqx_amd/libtmatch.so emqx_amd/variants/libtmatch_*.so; do
  name=$(basename $so .so)
  for d in ${DEFERS:-2 8 32 1000000000}; do
    for st in 1 3; do
      echo "== $name defer=$d streams=$st" >> $OUT/timing.txt
      TM_LIB=$so timeout -k 10 120 python3 -u tools/profile_walk.py --large-path one --lb-defer $d --streams $st "$@" 2>&1 | grep -v amdgpu.ids >> $OUT/timing.txt
    done
  done
done
