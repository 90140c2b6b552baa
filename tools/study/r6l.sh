set -e
A="--steps,20,--warmup,5,--no-cpu,--no-parity,--latency-batches,10"
bash tools/gpu.sh r6l bench:new1:$A export:TM_LIB=emqx_amd/variants/libtmatch_lockrel.so bench:old1:$A unset:TM_LIB bench:new2:$A export:TM_LIB=emqx_amd/variants/libtmatch_lockrel.so bench:old2:$A
