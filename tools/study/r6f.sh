set -e
bash tools/gpu.sh r6f smoke tests bench:bench_driver:--steps,20,--warmup,5 \
  export:TM_HOST_TIMING=1 bench:b_writes:--steps,20,--warmup,5,--latency-batches,0,--no-parity,--no-cpu
