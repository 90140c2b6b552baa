set -e
bash tools/gpu.sh r6g prof:--outputs,pairs bench:w64:--steps,20,--warmup,5,--latency-batches,0,--no-parity,--no-cpu,--route-writers,64 \
  bench:w16:--steps,20,--warmup,5,--latency-batches,0,--no-parity,--no-cpu,--route-writers,16
