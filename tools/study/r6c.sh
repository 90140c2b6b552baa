set -e
bash tools/gpu.sh r6c tests:pairs bench:bench_pairs:--steps,20,--warmup,5,--outputs,pairs,--latency-batches,0,--route-writers,0 \
  walk:--outputs,pairs walk:--outputs,csr walk:--order,sorted,--window,4096 walk:--order,sorted,--window,65536 walk:--order,sorted \
  export:TM_HOST_TIMING=1 bench:bench_writes:--steps,5,--warmup,1,--latency-batches,0,--no-parity
