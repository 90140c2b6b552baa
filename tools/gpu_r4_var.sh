#!/bin/bash
# Round 4 one-pass studies: every emqx_amd/variants build on the walk driver,
# one stream and three (bench.py's overlapped steps), on the one-pass path;
# the product library on the two-phase path for reference.
# usage: tools/gpu_r4_var.sh <tag> [profile_walk.py args]
set -e
TAG=$1; shift
OUT=gpurun_out/var_$TAG
mkdir -p $OUT
for st in 1 3; do
  echo "== product phases streams=$st" >> $OUT/timing.txt
  timeout -k 10 120 python3 -u tools/profile_walk.py --large-path phases --streams $st "$@" 2>&1 | grep -v amdgpu.ids >> $OUT/timing.txt
done
for so in emqx_amd/variants/libtmatch_*.so; do
  name=$(basename $so .so)
  for st in 1 3; do
    echo "== $name one streams=$st" >> $OUT/timing.txt
    TM_LIB=$so timeout -k 10 120 python3 -u tools/profile_walk.py --large-path one --streams $st "$@" 2>&1 | grep -v amdgpu.ids >> $OUT/timing.txt
  done
done
