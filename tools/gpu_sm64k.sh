#!/bin/bash
# One launch for batches up to 64k topics (study build sm64k) vs the product
# (one launch up to 8192): parity subset of the study build, then host-to-host
# latency at 4k-64k topics for both.  usage: tools/gpu_sm64k.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
TM_LIB=emqx_amd/variants/libtmatch_sm64k.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q \
  --timeout 300 --timeout-method thread -k "in_place or zero_copy or c3_reduced or random_sets or staging or mixed_batch or wave_walk_limits or c2_reduced or deep" > $OUT/parity_sm64k.log 2>&1
tail -1 $OUT/parity_sm64k.log
timeout -k 10 300 python3 -u tools/lat_sweep.py > $OUT/lat.jsonl 2> $OUT/lat.err
TM_LIB=emqx_amd/variants/libtmatch_sm64k.so timeout -k 10 300 python3 -u tools/lat_sweep.py >> $OUT/lat.jsonl 2>> $OUT/lat.err
