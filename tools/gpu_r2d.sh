mkdir -p gpurun_out/r2d
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "c3deep or levels_beyond or deep_topics or maximum_size or edge or churn" > gpurun_out/r2d/tests.log 2>&1; tail -3 gpurun_out/r2d/tests.log
timeout -k 10 120 ./tools/store_bench 4 > gpurun_out/r2d/store.csv 2>&1
timeout -k 10 400 python -u tools/bulk_deltas.py > gpurun_out/r2d/bulk.json 2> gpurun_out/r2d/bulk.err
cat gpurun_out/r2d/store.csv gpurun_out/r2d/bulk.json
bash tools/gpu_variants.sh r2e --batches 20
cat gpurun_out/var_r2e/timing.txt
