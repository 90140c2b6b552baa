set -e
B="--steps,20,--warmup,5,--latency-batches,0,--route-writers,0,--no-cpu,--no-parity"
bash tools/gpu.sh r6k tests walk:--config,c3deep,--outputs,pairs walk:--config,c3deep,--outputs,csr walk:--outputs,pairs \
  bench:c3deep:--config,c3deep,--warmup,5,--latency-batches,0,--route-writers,0,--no-cpu \
  bench:s3:$B bench:s2:$B,--streams,2 bench:s4:$B,--streams,4 \
  export:TM_HOST_TIMING=1 bench:full:--steps,20,--warmup,5,--no-cpu,--no-parity
