set -e
bash tools/gpu.sh r6close3 smoke tests prof:--outputs,pairs bench:bench_default bench:bench_driver:--steps,20,--warmup,5
