#!/bin/bash
# Phase timings of one-launch 4k batches (stamped study build, tools/mk_stamps.py).
# usage: tools/gpu_stamps.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
TM_LIB=emqx_amd/variants/libtmatch_stamps.so timeout -k 10 250 python3 -u tools/stamps_study.py > $OUT/stamps.log 2>&1
