#!/bin/bash
# Time experimental builds of libtmatch (emqx_amd/variants/*.so) on the walk
# driver, each after a short parity check.
# usage: tools/gpu_variants.sh <tag> [profile_walk.py args]
set -e
TAG=$1; shift
OUT=gpurun_out/var_$TAG
mkdir -p $OUT
for so in emqx_amd/variants/libtmatch_*.so; do
  name=$(basename $so .so)
  echo "== $name" >> $OUT/timing.txt
  [ -n "$NOTEST" ] || TM_LIB=$so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread -k "c3_reduced or random_sets or c1_full or edge or deep or first_batch or c2_reduced" \
    > $OUT/tests_$name.log 2>&1 || { echo "PARITY FAILED" >> $OUT/timing.txt; continue; }
  TM_LIB=$so timeout -k 10 120 python3 -u tools/profile_walk.py "$@" 2>&1 | grep -v amdgpu.ids >> $OUT/timing.txt
done
