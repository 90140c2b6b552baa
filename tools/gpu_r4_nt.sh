#!/bin/bash
# Round 4 study: non-temporal vocab / exact-key loads in the walk (tools/study/mk_nt.py).
set -e
OUT=gpurun_out/nt_$1
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in prod nt_f nt_e nt_x; do
    lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
    echo "== $v $rep" >> $OUT/walk.txt
    TM_LIB=$lib timeout -k 10 120 python3 -u tools/profile_walk.py --config c3 --large-path phases --streams 1 --batches 24 2>&1 \
      | grep -v amdgpu.ids >> $OUT/walk.txt
  done
done
for v in prod nt_f nt_e nt_x; do
  lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
  TM_LIB=$lib timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_$v -o run --output-format csv -- \
    python3 -u tools/profile_walk.py --config c3 --batches 8 > $OUT/pmc_$v.log 2>&1
done
echo done > $OUT/done.txt
