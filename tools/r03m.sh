# round-3 session: the whole GPU suite (noscan path for small batches), smoke, full bench
bash tools/gpu.sh r03m tests || exit 1
bash tools/gpu.sh r03m smoke || exit 1
BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh r03m bench
