#!/bin/bash
# End-of-session GPU check: the whole GPU suite, smoke(), the matches_filter
# benchmark, then the profile of the default bench (kernel traces + PMC
# passes that restamp profiles/pmc_c3.json through tools/prof_report.py).
set -e
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
tail -2 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python -u tools/mf_bench.py > $O/mf_bench.json 2> $O/mf_bench.err
bash tools/gpu_prof.sh r2f --config c3 --batches 8
