#!/bin/bash
# Round 4: one-pass parked-path tests + trace + defer sweep, then the ITAB study.
set -e
export TMPDIR=/tmp
O=gpurun_out/one3
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "one_pass or parked or lookback" > $O/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof0 -o run --output-format csv -- \
  python3 tools/profile_walk.py --large-path one --lb-defer 0 --streams 1 --config c3 --batches 24 > $O/prof0.log 2>&1
for d in 0 16 64 1000000000; do
  timeout -k 10 120 python3 tools/profile_walk.py --large-path one --lb-defer $d --streams 1 --config c3 --batches 24 2>&1 \
    | grep -v amdgpu.ids >> $O/timing.txt
done
bash tools/gpu_r4_itab.sh a "prod:emqx_amd/libtmatch.so:" "itab2:emqx_amd/variants/libtmatch_itab.so:2" \
  "itabns2:emqx_amd/variants/libtmatch_itab_ns.so:2" "itab23:emqx_amd/variants/libtmatch_itab.so:2,3" \
  "itab12:emqx_amd/variants/libtmatch_itab.so:1,2"
