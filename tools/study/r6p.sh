set -e
V=emqx_amd/variants/libtmatch_pairs_direct.so
bash tools/gpu.sh r6p walk:--outputs,pairs export:TM_LIB=$V walk:--outputs,pairs unset:TM_LIB walk:--outputs,pairs export:TM_LIB=$V walk:--outputs,pairs \
  bench:direct:--steps,20,--warmup,5,--latency-batches,0,--route-writers,0,--no-cpu unset:TM_LIB bench:product:--steps,20,--warmup,5,--latency-batches,0,--route-writers,0,--no-cpu
