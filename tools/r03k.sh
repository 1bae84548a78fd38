# round-3 session: parity after the scan poll / tx state changes, scatter and tx timing, full bench, c3 stream shapes
TESTS="tests/test_gpu_scatter.py tests/test_gpu_volume.py tests/test_gpu_tx.py tests/test_gpu_parity.py" bash tools/gpu.sh r03k tests || exit 1
SCB_CFGS="c5 c2" bash tools/gpu.sh r03k scb || exit 1
TXB_ARGS="1048576 40 1 --rotate 6" bash tools/gpu.sh r03k txbench || exit 1
BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh r03k bench || exit 1
mv gpurun_out/r03k/bench.log gpurun_out/r03k/bench_full.log
BENCH_ARGS="--config c3 --queues 4 --streams 4 --steps 40 --warmup 5 --no-cpu-baseline --no-extra" bash tools/gpu.sh r03k bench || exit 1
mv gpurun_out/r03k/bench.log gpurun_out/r03k/bench_c3_s4.log
