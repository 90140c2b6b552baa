#!/bin/bash
# Final round-3 check on one box: GPU suite, smoke(), then the profile that
# restamps profiles/pmc_c3.json (tools/gpu_prof.sh).  usage: tools/gpu_final3.sh <tag>
set -e
OUT=gpurun_out/final_$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
tail -1 $OUT/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash tools/gpu_prof.sh $1
