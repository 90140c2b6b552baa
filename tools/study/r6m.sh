set -e
A="--steps,20,--warmup,5,--no-cpu,--no-parity,--latency-batches,10"
bash tools/gpu.sh r6m bench:base:$A bench:cf50:$A,--commit-first,50 bench:tk:$A,--small-ticket,1 bench:base2:$A bench:cf200:$A,--commit-first,200 bench:tk2:$A,--small-ticket,1
