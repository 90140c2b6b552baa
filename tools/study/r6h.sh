set -e
A="--steps,5,--warmup,2,--no-parity,--no-cpu,--route-writers,0,--latency-batches,10"
bash tools/gpu.sh r6h bench:c1:$A export:TM_STUDY_NODRAIN=1 bench:nodrain:$A unset:TM_STUDY_NODRAIN bench:c2:$A
