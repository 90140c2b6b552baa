set -e
bash tools/gpu.sh r6j tests:pairs walk:--config,c3deep,--outputs,pairs walk:--config,c3deep,--outputs,csr \
  bench:c3deep:--config,c3deep,--warmup,5,--latency-batches,0,--route-writers,0,--no-cpu
