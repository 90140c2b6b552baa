set -e
bash tools/gpu.sh r6d walk:--outputs,pairs export:TM_STUDY_PAIRS=1 walk:--outputs,pairs export:TM_STUDY_PAIRS=2 walk:--outputs,pairs unset:TM_STUDY_PAIRS \
  bench:w5:--steps,20,--warmup,5,--latency-batches,0,--route-writers,0,--no-cpu \
  bench:w100:--steps,20,--warmup,100,--latency-batches,0,--route-writers,0,--no-cpu \
  bench:w5b:--steps,20,--warmup,5,--latency-batches,0,--route-writers,0,--no-cpu
