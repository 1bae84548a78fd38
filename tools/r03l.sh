# round-3 session: bench c5 twice (variance), the HBM streaming floor of the access pattern, group/daemon tests
B="--steps 40 --warmup 5 --no-cpu-baseline --no-extra"
BENCH_ARGS="$B" bash tools/gpu.sh r03l bench || exit 1; mv gpurun_out/r03l/bench.log gpurun_out/r03l/bench1.log
BENCH_ARGS="$B" bash tools/gpu.sh r03l bench || exit 1; mv gpurun_out/r03l/bench.log gpurun_out/r03l/bench2.log
timeout -k 10 120 build/hbm_floor 8388608 50 > gpurun_out/r03l/hbm_floor.log 2>&1 || exit 1
TESTS="tests/test_gpu_group.py tests/test_daemon_gpu.py tests/test_gpu_multiproc.py tests/test_gpu_bench.py" bash tools/gpu.sh r03l tests
