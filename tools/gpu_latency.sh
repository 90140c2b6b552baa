#!/bin/bash
# Host-batch latency (tools/latency_trace.py) of the product library and of
# every study variant under emqx_amd/variants/, at a few batch sizes.
# usage: tools/gpu_latency.sh <tag> [batch sizes...]
set -e
TAG=$1; shift
SIZES=${@:-"4096 16384 65536"}
OUT=gpurun_out/lat_$TAG
mkdir -p $OUT
for so in emqx_amd/libtmatch.so emqx_amd/variants/libtmatch_*.so; do
  [ -f $so ] || continue
  name=$(basename $so .so)
  for b in $SIZES; do
    TM_LIB=$so timeout -k 10 120 python3 -u tools/latency_trace.py --batch $b --reps 60 2>&1 \
      | grep -v amdgpu.ids | sed "s/^/$name /" >> $OUT/latency.txt
  done
done
TM_HOST_TIMING=1 timeout -k 10 120 python3 -u tools/latency_trace.py --batch 65536 --reps 30 > $OUT/host_timing.txt 2>&1
