set -e
bash tools/gpu.sh r6e tests:pairs walk:--outputs,pairs walk:--outputs,csr \
  bench:b_pairs:--steps,20,--warmup,5,--outputs,pairs,--latency-batches,0,--route-writers,0,--no-cpu \
  bench:b_csr:--steps,20,--warmup,5,--latency-batches,0,--route-writers,0,--no-cpu \
  export:TM_HOST_TIMING=1 bench:b_writes:--steps,20,--warmup,5,--latency-batches,0,--no-parity
