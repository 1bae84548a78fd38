#!/bin/bash
# Round-3 GPU sessions (each a sequence of tools/gpu.sh steps):
#   bash tools/r03.sh <session>   output under gpurun_out/<session>/
set -o pipefail
S=${1:?session}
case $S in
  r03i)
    # round-3 session: parity of the scan/base change and the tx fast path,
    # scan chunks-per-thread A/B, c3 LDS-DMA A/B, tx timing on rotating buffers
    TESTS="tests/test_gpu_scatter.py tests/test_gpu_volume.py tests/test_gpu_parity.py tests/test_gpu_tx.py tests/test_gpu_group.py" bash tools/gpu.sh r03i tests || exit 1
    for k in 4 2 1; do
      USN_SCAN_CPT=$k SCB_CFGS="c5 c2" bash tools/gpu.sh r03i scb || exit 1
      mv gpurun_out/r03i/scb_c5.log gpurun_out/r03i/scb_c5_cpt$k.log
      mv gpurun_out/r03i/scb_c2.log gpurun_out/r03i/scb_c2_cpt$k.log
    done
    TXB_ARGS="1048576 40 1 --rotate 6" bash tools/gpu.sh r03i txbench || exit 1
    ABL_CFGS=c3 ABL_VARIANTS="base c3glds" bash tools/gpu.sh r03i abl
    ;;
  r03j)
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
    ;;
  r03k)
    # round-3 session: parity after the scan poll / tx state changes, scatter and tx timing, full bench, c3 stream shapes
    TESTS="tests/test_gpu_scatter.py tests/test_gpu_volume.py tests/test_gpu_tx.py tests/test_gpu_parity.py" bash tools/gpu.sh r03k tests || exit 1
    SCB_CFGS="c5 c2" bash tools/gpu.sh r03k scb || exit 1
    TXB_ARGS="1048576 40 1 --rotate 6" bash tools/gpu.sh r03k txbench || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh r03k bench || exit 1
    mv gpurun_out/r03k/bench.log gpurun_out/r03k/bench_full.log
    BENCH_ARGS="--config c3 --queues 4 --streams 4 --steps 40 --warmup 5 --no-cpu-baseline --no-extra" bash tools/gpu.sh r03k bench || exit 1
    mv gpurun_out/r03k/bench.log gpurun_out/r03k/bench_c3_s4.log
    ;;
  r03l)
    # round-3 session: bench c5 twice (variance), the HBM streaming floor of the access pattern, group/daemon tests
    B="--steps 40 --warmup 5 --no-cpu-baseline --no-extra"
    BENCH_ARGS="$B" bash tools/gpu.sh r03l bench || exit 1; mv gpurun_out/r03l/bench.log gpurun_out/r03l/bench1.log
    BENCH_ARGS="$B" bash tools/gpu.sh r03l bench || exit 1; mv gpurun_out/r03l/bench.log gpurun_out/r03l/bench2.log
    timeout -k 10 120 build/hbm_floor 8388608 50 > gpurun_out/r03l/hbm_floor.log 2>&1 || exit 1
    TESTS="tests/test_gpu_group.py tests/test_daemon_gpu.py tests/test_gpu_multiproc.py tests/test_gpu_bench.py" bash tools/gpu.sh r03l tests
    ;;
  r03m)
    # round-3 session: the whole GPU suite (noscan path for small batches), smoke, full bench
    bash tools/gpu.sh r03m tests || exit 1
    bash tools/gpu.sh r03m smoke || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh r03m bench
    ;;
  r03n)
    # round-3 session: kernel breakdown of the bench (all configs) and of the tx
    # rings; A/B of the scatter's grouped write-out
    SCB_CFGS="c5 c2" SCB_VARIANTS="base scg0" bash tools/gpu.sh r03n scb || exit 1
    bash tools/gpu.sh r03n rocprof || exit 1
    TXB_ARGS="1048576 24 1 --rotate 6" bash tools/gpu.sh r03n txprof
    ;;
  r03o)
    # round-3 session: scan chunks-per-thread A/B after the poll change; PMC traffic of the final kernels
    O=gpurun_out/r03o
    for k in 4 2; do
      USN_SCAN_CPT=$k SCB_CFGS="c5" bash tools/gpu.sh r03o scb || exit 1
      mv $O/scb_c5.log $O/scb_c5_cpt$k.log
    done
    PMC_CFGS="c5 c2 c4 c3" bash tools/gpu.sh r03o pmc || exit 1
    TXB_ARGS="1048576 24 1 --rotate 6" bash tools/gpu.sh r03o txpmc || exit 1
    python3 tools/pmc_traffic.py $O/txpmcf $O/txpmcw 1048576 $O/pmc_c4tx.json > $O/pmct_c4tx.log 2>&1
    ;;
  r03p)
    # round-3 session: scatter chunk length A/B (c5/c2 through scatter_bench, tx
    # rings through txbench); c5 calls of 4 and 8 rings
    O=gpurun_out/r03p
    mkdir -p $O
    for k in 8 4; do
      USN_SCATTER_TC=$k SCB_CFGS="c5 c2" bash tools/gpu.sh r03p scb || exit 1
      mv $O/scb_c5.log $O/scb_c5_tc$k.log; mv $O/scb_c2.log $O/scb_c2_tc$k.log
    done
    for k in 1 4 8; do
      USN_SCATTER_TC=$k TXB_ARGS="1048576 30 1 --rotate 6" bash tools/gpu.sh r03p txbench || exit 1
      mv $O/txbench.log $O/txbench_tc$k.log
    done
    B="--steps 30 --warmup 5 --no-cpu-baseline --no-extra"
    for q in 2 4 8; do
      BENCH_ARGS="$B --queues $q --rings-per-launch $q" bash tools/gpu.sh r03p bench || exit 1
      mv $O/bench.log $O/bench_q$q.log
    done
    ;;
  r03q)
    # round-3 final check of the tree: the whole GPU suite, smoke, the default
    # bench line, and a rocprof of the default bench
    bash tools/gpu.sh r03q tests || exit 1
    bash tools/gpu.sh r03q smoke || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh r03q bench || exit 1
    bash tools/gpu.sh r03q rocprof
    ;;
  r03r)
    # round-3 session: c3 launch shapes (host-enqueue bound at 2 rings per call on
    # 2 streams: 17-28 Gpkt/s between runs), HIP API times of the c3 bench
    O=gpurun_out/r03r
    mkdir -p $O
    B="--config c3 --steps 40 --warmup 5 --no-cpu-baseline --no-extra"
    for v in "4 2 2" "4 4 1" "8 8 1" "8 4 2"; do
      set -- $v
      BENCH_ARGS="$B --queues $1 --rings-per-launch $2 --streams $3" bash tools/gpu.sh r03r bench || exit 1
      mv $O/bench.log $O/bench_q$1_p$2_s$3.log
    done
    rm -rf $O/rt
    timeout -k 10 300 rocprofv3 --runtime-trace --stats --output-format csv -d $O/rt -o run -- \
      python3 bench.py $B --queues 4 --launch-probe 20 --ramp 20 > $O/rt.log 2>&1 || exit 1
    ;;
  r03s)
    # round-3 session: u8 count rows (255 escapes to a u16 row): parity incl.
    # the escape cases, scan + scatter timing, the default bench
    TESTS="tests/test_gpu_scatter.py tests/test_gpu_volume.py tests/test_gpu_parity.py tests/test_gpu_tx.py" bash tools/gpu.sh r03s tests || exit 1
    SCB_CFGS="c5 c2" bash tools/gpu.sh r03s scb || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh r03s bench
    ;;
  r03t)
    # round-3 session: A/B of the u8 count rows against the u16 ones (build/abl/u16 =
    # the tree before them), whole calls interleaved in one process, and scan +
    # scatter alone; c4's DROP bin escapes in every tile
    O=gpurun_out/r03t
    mkdir -p $O
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --batches 4 --multi 2 --rounds 5 --launches 40" ABL_VARIANTS="u8 u16" bash tools/gpu.sh r03t abl || exit 1
    ABL_CFGS="c4 c2" ABL_ARGS="--frames 1048576 --batches 16 --multi 8 --rounds 5 --launches 40" ABL_VARIANTS="u8 u16" bash tools/gpu.sh r03t abl || exit 1
    for c in c5 c4 c2; do
      if [ $c = c5 ]; then A="--frames 8388608 --multi 2"; else A="--frames 1048576 --multi 8"; fi
      timeout -k 10 300 python tools/scatter_bench.py --config $c $A --json $O/scb_$c.json u8 u16 u8 u16 > $O/scb_$c.log 2>&1 || exit 1
    done
    ;;
  r03u)
    # round-3 session: the tree after the u8 A/B (u16 rows), the whole GPU suite,
    # smoke, the default bench line (c3 in its new shape), c5 at one ring per call
    O=gpurun_out/r03u
    mkdir -p $O
    bash tools/gpu.sh r03u tests || exit 1
    bash tools/gpu.sh r03u smoke || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh r03u bench || exit 1
    mv $O/bench.log $O/bench_full.log
    B="--steps 40 --warmup 5 --no-cpu-baseline --no-extra"
    HOSTIO_ARGS="c2 1048576 8 4 6" bash tools/gpu.sh r03u hostio || exit 1
    mv $O/hostio.log $O/hostio_c2.log
    HOSTIO_ARGS="c5 1048576 8 4 6" bash tools/gpu.sh r03u hostio || exit 1
    mv $O/hostio.log $O/hostio_c5.log
    for s in 1 2; do
      BENCH_ARGS="$B --queues 2 --rings-per-launch 1 --streams $s" bash tools/gpu.sh r03u bench || exit 1
      mv $O/bench.log $O/bench_p1_s$s.log
    done
    ;;
  r03v)
    # round-3 session: the scan at 8 bins per lane (16-byte loads, USN_SCAN_LW=8):
    # parity with it, scan + scatter A/B against 4 bins per lane, bench with it;
    # the PCIe-inclusive loop with the lists (hostio.py, ABI v3)
    O=gpurun_out/r03v
    mkdir -p $O
    USN_SCAN_LW=8 TESTS="tests/test_gpu_scatter.py tests/test_gpu_volume.py tests/test_gpu_parity.py" bash tools/gpu.sh r03v tests || exit 1
    for k in 4 8 4 8; do
      USN_SCAN_LW=$k SCB_CFGS="c5" bash tools/gpu.sh r03v scb || exit 1
      cat $O/scb_c5.log >> $O/scb_c5_lw$k.log
    done
    B="--steps 40 --warmup 5 --no-cpu-baseline --no-extra"
    for k in 4 8; do
      USN_SCAN_LW=$k BENCH_ARGS="$B" bash tools/gpu.sh r03v bench || exit 1
      mv $O/bench.log $O/bench_lw$k.log
    done
    HOSTIO_ARGS="c2 1048576 8 4 6" bash tools/gpu.sh r03v hostio || exit 1
    mv $O/hostio.log $O/hostio_c2.log
    HOSTIO_ARGS="c5 1048576 8 4 6" bash tools/gpu.sh r03v hostio || exit 1
    mv $O/hostio.log $O/hostio_c5.log
    ;;
  r03w)
    # round-3 session: where the tx ring's time goes now (phase stamps of the tx
    # kernel, the launch without rule probes) and the c5 classify's phases
    O=gpurun_out/r03w
    mkdir -p $O
    timeout -k 10 300 python tools/stamps.py c4tx 1048576 > $O/stamps_c4tx.log 2>&1 || exit 1
    timeout -k 10 300 python tools/stamps.py c5 8388608 > $O/stamps_c5.log 2>&1 || exit 1
    for v in base txnoprobe base txnoprobe; do
      timeout -k 10 300 python tools/txbench.py 1048576 30 1 build/abl/$v/libusn.so --rotate 6 >> $O/txbench_$v.log 2>&1 || exit 1
    done
    ;;
  r03x)
    # round-3 session: phase stamps of the tx kernel and the c5 classify (the
    # 512-thread build's buffer)
    O=gpurun_out/r03x
    mkdir -p $O
    timeout -k 10 300 python tools/stamps.py c4tx 1048576 > $O/stamps_c4tx.log 2>&1 || exit 1
    timeout -k 10 300 python tools/stamps.py c5 8388608 > $O/stamps_c5.log 2>&1 || exit 1
    ;;
  r03y)
    # round-3 session: a batch keeps its classify-time bins through usn_finalize
    # (endpoints added in between); the whole GPU suite and smoke on the tree
    bash tools/gpu.sh r03y tests || exit 1
    bash tools/gpu.sh r03y smoke
    ;;
  r03z)
    # round-3 session: the tx probes' slot reads non-temporal (USN_TX_SLOT_NT,
    # build/abl/txslotnt) against the default, alternating, on rotating buffers
    O=gpurun_out/r03z
    mkdir -p $O
    for v in base txslotnt base txslotnt; do
      timeout -k 10 300 python tools/txbench.py 1048576 30 1 build/abl/$v/libusn.so --rotate 6 > $O/tmp.log 2>&1 || exit 1
      grep '^{"n"' $O/tmp.log >> $O/txbench_$v.log
    done
    ;;
  r03f)
    # round-3 final tree: the default bench line (as the driver runs it) and a
    # rocprof of the bench
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh r03f bench || exit 1
    bash tools/gpu.sh r03f rocprof
    ;;
  *) echo "unknown session $S"; exit 2 ;;
esac
