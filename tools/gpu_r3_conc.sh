#!/bin/bash
# Concurrent callers: GPU suite, then kernel traces of 4 native caller threads
# (no churn) and plain runs at 1, 4 and 16 threads.
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "notest" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
fi
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/p4 -o run -- \
  python3 -u tools/callers_trace.py --threads 4 > $OUT/p4.log 2>&1
for t in 1 4 16; do
  timeout -k 10 200 python3 -u tools/callers_trace.py --threads $t --seconds 1 >> $OUT/plain.log 2>&1
done
TM_LIB=emqx_amd/variants/libtmatch_stamps.so timeout -k 10 250 python3 -u tools/stamps_study.py > $OUT/stamps.log 2>&1
