set -e
O=gpurun_out/s3c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
tail -2 $O/gputest.log
NOTEST=1 bash tools/gpu_variants.sh wide --config c3 --batches 12
PASSES="FETCH_SIZE;TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" bash tools/gpu_libs_prof.sh wide emqx_amd/variants/libtmatch_a_nowide.so emqx_amd/variants/libtmatch_b_wide256.so emqx_amd/variants/libtmatch_c_wide128.so -- --config c3 --batches 8
