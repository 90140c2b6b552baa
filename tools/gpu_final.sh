set -e
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
tail -2 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/gpu_prof.sh r2d --config c3 --batches 8
