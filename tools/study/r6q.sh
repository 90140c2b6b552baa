set -e
V=emqx_amd/variants/libtmatch_prev_close.so
B="--steps,20,--warmup,5,--latency-batches,0,--route-writers,0,--no-cpu"
bash tools/gpu.sh r6q tests:pairs walk:--outputs,pairs export:TM_LIB=$V walk:--outputs,pairs unset:TM_LIB walk:--outputs,pairs export:TM_LIB=$V walk:--outputs,pairs unset:TM_LIB \
  bench:new1:$B export:TM_LIB=$V bench:old1:$B unset:TM_LIB bench:new2:$B export:TM_LIB=$V bench:old2:$B unset:TM_LIB \
  walk:--config,c2,--outputs,pairs walk:--config,c3deep,--outputs,pairs
