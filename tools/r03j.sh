# round-3 session: c5 bench launch shapes (one stream; the scatter on the side
# stream; two streams of one 2-ring launch each), PMC traffic of c5/c2/c4 and
# of the tx call, rocprof of the default bench
B="--steps 40 --warmup 5 --no-cpu-baseline --no-extra"
O=gpurun_out/r03j
BENCH_ARGS="$B" bash tools/gpu.sh r03j bench || exit 1; mv $O/bench.log $O/bench_default.log
BENCH_ARGS="$B --lists-async 1" bash tools/gpu.sh r03j bench || exit 1; mv $O/bench.log $O/bench_async.log
BENCH_ARGS="$B --streams 2 --queues 4 --rings-per-launch 2" bash tools/gpu.sh r03j bench || exit 1; mv $O/bench.log $O/bench_s2.log
PMC_CFGS="c5 c2 c4" bash tools/gpu.sh r03j pmc || exit 1
TXB_ARGS="1048576 24 1 --rotate 6" bash tools/gpu.sh r03j txpmc || exit 1
python3 tools/pmc_traffic.py $O/txpmcf $O/txpmcw 1048576 $O/pmc_c4tx.json > $O/pmct_c4tx.log 2>&1
bash tools/gpu.sh r03j rocprof
