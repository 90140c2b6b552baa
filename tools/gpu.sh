#!/bin/bash
# One parametrised GPU-box runner (replaces the per-study gpu_*.sh recipes).
# Every step runs under its own time limit; the first failing or timed-out
# step ends the script (set -e: no retries, nothing more on the GPU after it).
#
# usage: tools/gpu.sh <tag> <step> [<step> ...]
#   smoke                     __graft_entry__.smoke()
#   tests[:<pytest -k expr>]  pytest -m gpu (verbose, per-test timeout; '+' in the
#                             expression stands for a space)
#   bench[:<name>:<args>]     bench.py <args> -> <name>.json (args: comma separated)
#   prof[:<profile_walk args>]  rocprofv3 --kernel-trace --stats over bench.py
#                             defaults + tools/profile_walk.py, then the PMC
#                             passes (one rocprofv3 --pmc run per group)
#   walk[:<args>]             tools/profile_walk.py <args> (isolated walk timing)
#   py:<name>:<script args>   python3 -u <script args> -> <name>.txt
#   export:<VAR>=<value>      set an environment variable for the steps after it
#                             (e.g. TM_LIB=emqx_amd/variants/libtmatch_<study>.so)
#   unset:<VAR>
# Output: gpurun_out/<tag>/
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n+1))
  kind=${step%%:*}
  rest=""; [ "$kind" != "$step" ] && rest=${step#*:}
  echo "[$(date +%T)] step $n: $step"
  case $kind in
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      tail -1 "$OUT/smoke.log" ;;
    tests)
      if [ -n "$rest" ]; then KARG=(-k "${rest//+/ }"); else KARG=(); fi
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        "${KARG[@]}" > "$OUT/tests_$n.log" 2>&1
      tail -2 "$OUT/tests_$n.log" ;;
    bench)
      name=${rest%%:*}; args=""; [ "$name" != "$rest" ] && args=${rest#*:}
      [ -z "$name" ] && name=bench
      timeout -k 10 500 python3 -u bench.py ${args//,/ } > "$OUT/$name.json" 2> "$OUT/$name.err"
      cut -c1-400 "$OUT/$name.json" ;;
    walk)
      timeout -k 10 300 python3 -u tools/profile_walk.py ${rest//,/ } > "$OUT/walk_$n.txt" 2>&1
      tail -5 "$OUT/walk_$n.txt" ;;
    py)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 600 python3 -u ${args//,/ } > "$OUT/$name.txt" 2>&1
      tail -5 "$OUT/$name.txt" ;;
    prof)
      mkdir -p "$OUT/prof"
      timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof/bench" -o run --output-format csv -- \
        python3 -u bench.py > "$OUT/prof/bench.json" 2> "$OUT/prof/bench.err"
      gzip -f "$OUT/prof/bench/run_kernel_trace.csv"
      timeout -k 10 200 python3 -u tools/profile_walk.py ${rest//,/ } > "$OUT/prof/timing.txt" 2>&1
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof/trace" -o run --output-format csv -- \
        python3 -u tools/profile_walk.py ${rest//,/ } > "$OUT/prof/trace.log" 2>&1
      i=0
      for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
                 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
                 "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
                 "GRBM_GUI_ACTIVE GRBM_COUNT"; do
        i=$((i+1))
        timeout -k 10 -s KILL 120 rocprofv3 --pmc $pmc -d "$OUT/prof/pmc$i" -o run --output-format csv -- \
          python3 -u tools/profile_walk.py ${rest//,/ } > "$OUT/prof/pmc$i.log" 2>&1
      done ;;
    export) export "$rest"; echo "  $rest" ;;
    unset) unset "$rest" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$(date +%T)] done" > "$OUT/done.txt"
