set -e
A="--warmup,5,--latency-batches,0,--route-writers,0"
bash tools/gpu.sh r6i2 bench:c1:--config,c1,$A bench:c2:--config,c2,$A bench:c2nm:--config,c2nm,$A bench:c3deep:--config,c3deep,$A bench:c5:--config,c5,$A
