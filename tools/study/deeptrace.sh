set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r5_deeptrace
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_deeptrace/new -o run --output-format csv -- python3 -u tools/profile_walk.py --config c3deep > gpurun_out/r5_deeptrace/new.log 2>&1
export TM_LIB=emqx_amd/variants/libtmatch_head.so
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_deeptrace/head -o run --output-format csv -- python3 -u tools/profile_walk.py --config c3deep > gpurun_out/r5_deeptrace/head.log 2>&1
