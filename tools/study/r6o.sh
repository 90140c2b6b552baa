set -e
A="--steps,20,--warmup,5,--no-cpu,--no-parity,--route-writers,0,--latency-batches,10"
bash tools/gpu.sh r6o bench:s0a:$A bench:s50a:$A,--cmb-spin,50 bench:s200a:$A,--cmb-spin,200 bench:s0b:$A bench:s50b:$A,--cmb-spin,50 bench:s200b:$A,--cmb-spin,200
