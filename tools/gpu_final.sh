set -e
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
tail -2 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python -u bench.py --config c3deep --no-cpu --concurrency 0 > $O/c3deep.json 2> $O/c3deep.err
bash tools/gpu_prof.sh r2e --config c3 --batches 8
