set -e
A="--steps,20,--warmup,5,--no-cpu,--no-parity,--route-writers,0,--latency-batches,10"
bash tools/gpu.sh r6n bench:l4a:$A,--combine-leaders,4 bench:l2a:$A,--combine-leaders,2 bench:l3a:$A,--combine-leaders,3 \
  bench:l4b:$A,--combine-leaders,4 bench:l2b:$A,--combine-leaders,2 bench:l3b:$A,--combine-leaders,3 \
  export:TM_BENCH_DIST_BACKEND=gloo \
  py:n2:-m,torch.distributed.run,--nnodes=1,--nproc-per-node=2,--master-addr=127.0.0.1,--master-port=29511,bench.py,--gpus,2,--steps,20,--warmup,5,--latency-batches,0,--route-writers,0,--no-cpu
