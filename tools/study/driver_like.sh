set -e
mkdir -p gpurun_out/r5_driver
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5_driver/gpu_tests.log 2>&1
tail -2 gpurun_out/r5_driver/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_driver/smoke.log 2>&1
tail -1 gpurun_out/r5_driver/smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5_driver/bench.json 2> gpurun_out/r5_driver/bench.err
cut -c1-300 gpurun_out/r5_driver/bench.json
