#!/bin/bash
# Round 6 GPU sessions (one tag per gpurun call; outputs under gpurun_out/<tag>/).
#   tools/r06.sh TAG
# The sessions are records: the A/B builds they time (build/abl/<name>) were
# built for them at the time, and the knobs behind r06m-r06p's priority
# variants and r06t's tx buffer loads have since left the source.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=${1:?tag}
export TMPDIR=/tmp
C3="--frames 262144 --multi 4 --batches 16 --streams 2 --rounds 5 --launches 60"
C2="--frames 1048576 --multi 8 --batches 16 --streams 2 --rounds 5 --launches 40"
C5="--frames 8388608 --multi 2 --batches 4 --rounds 5 --launches 30"
case $S in
  r06b)
    # ADVICE r05 (release waits), then what a call's rx completion event and
    # host-mapped state gather cost: one test-build binary,
    # knobs per context, interleaved in one process, c3 / c2 / c5 call shapes
    TESTS=tests/test_gpu_release.py bash tools/gpu.sh $S tests || exit 1
    V="product testlib@USN_RX_EV=1 testlib@USN_RX_EV=0 testlib@USN_RX_EV=2 testlib@USN_RX_EV=3 testlib@USN_RX_STATE=0 testlib@USN_RX_EV=0,USN_RX_STATE=0"
    ABL_CFGS=c3 ABL_ARGS="$C3" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c2 ABL_ARGS="$C2" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c5 ABL_ARGS="$C5" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    BENCH_ARGS="--steps 20 --warmup 3 --extras c3 --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    ;;
  r06c)
    # the cheaper probe hash (24-bit multiplies, no h2 finaliser), 32-bit header
    # addresses, branch-free pidx: the suite (new image hashes), then the
    # product against the previous commit (build/abl/r06old) and the rx
    # completion event bound to the scatter's dispatch (USN_RX_EV=4)
    bash tools/gpu.sh $S tests || exit 1
    V="product r06old testlib@USN_RX_EV=4 testlib@USN_RX_EV=0"
    ABL_CFGS=c5 ABL_ARGS="$C5" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c3 ABL_ARGS="$C3" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c2 ABL_ARGS="$C2" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c4 ABL_ARGS="$C2" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    # the tx grid (8 rings per launch, 8 rotating buffers): previous commit, product, twice
    for v in old new old new; do
      L=""; [ $v = old ] && L=build/abl/r06old/libusn.so
      TAILN=3 TXB_ARGS="1048576 24 1 $L --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    BENCH_ARGS="--steps 20 --warmup 3 --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    ;;
  r06d)
    # the completion event bound to the scatter's dispatch by default (rx and
    # tx): the suite; the tx grid against the hash A/B builds (which of the
    # two hash changes slowed r06c's tx grid); c3 / c2 calls against mode 1
    bash tools/gpu.sh $S tests || exit 1
    for v in new r06old oldkey oldmac oldboth new r06old oldkey oldmac oldboth; do
      L=""; [ $v != new ] && L=build/abl/$v/libusn.so
      TAILN=1 TXB_ARGS="1048576 24 1 $L --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    V="product testlib@USN_RX_EV=1 testlib@USN_RX_EV=0"
    ABL_CFGS=c3 ABL_ARGS="$C3" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c2 ABL_ARGS="$C2" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    BENCH_ARGS="--steps 20 --warmup 3 --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    ;;
  r06e)
    # MAC hash reverted, completion events bound for launches <= 2048 tiles:
    # the suite; c5's U geometry (a smaller displacement copy per tile: lower
    # slot load, larger groups); c3 / c2 against recorded events; the tx grid
    bash tools/gpu.sh $S tests || exit 1
    V="product testlib@USN_PH_LOAD=0.35,USN_PH_GROUP=16 testlib@USN_PH_LOAD=0.4,USN_PH_GROUP=14 testlib@USN_PH_LOAD=0.3,USN_PH_GROUP=20 testlib@USN_PH_LOAD=0.25,USN_PH_GROUP=26"
    ABL_CFGS=c5 ABL_ARGS="$C5" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    V="product testlib@USN_RX_EV=1"
    ABL_CFGS=c3 ABL_ARGS="$C3" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c2 ABL_ARGS="$C2" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    for v in new new; do
      TAILN=1 TXB_ARGS="1048576 24 1 --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    BENCH_ARGS="--steps 20 --warmup 3 --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    ;;
  r06f)
    # the tx EARLY look-back over packed words (one 16-byte load per thread
    # instead of 2048 granule lines per tile): the tx tests, then the tx grid
    # against HEAD~ (build/abl/r06prev), interleaved; the bench's new probe
    TESTS="tests/test_gpu_tx.py tests/test_gpu_parity.py" bash tools/gpu.sh $S tests || exit 1
    for v in new r06prev new r06prev new r06prev; do
      L=""; [ $v != new ] && L=build/abl/$v/libusn.so
      TAILN=1 TXB_ARGS="1048576 24 1 $L --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    for v in new r06prev; do
      L=""; [ $v != new ] && L=build/abl/$v/libusn.so
      TAILN=1 TXB_ARGS="1048576 24 1 $L --rotate 8 --rings 1" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench1_${v}_$RANDOM.log
    done
    BENCH_ARGS="--steps 20 --warmup 3 --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    ;;
  r06g)
    # where an 8-ring tx grid's tile time goes now (stamps, the diagnostic
    # build), and the kernels of the bench in rocprof
    STAMP_ARGS="c4tx 1048576 8" bash tools/gpu.sh $S stamps || exit 1
    mv gpurun_out/$S/stamps.log gpurun_out/$S/stamps_c4tx8.log
    STAMP_ARGS="c4tx 1048576 1" bash tools/gpu.sh $S stamps || exit 1
    mv gpurun_out/$S/stamps.log gpurun_out/$S/stamps_c4tx1.log
    STAMP_ARGS="c5 8388608" bash tools/gpu.sh $S stamps || exit 1
    mv gpurun_out/$S/stamps.log gpurun_out/$S/stamps_c5.log
    bash tools/gpu.sh $S rocprof || exit 1
    ;;
  r06h)
    # tile_prefix_max with one barrier (two calls per tx tile) and the rx
    # classify at two tiles per workgroup (TM_DISPLDS, the second tile's loads
    # prefetched): the suite; c5 / c4 against one tile per workgroup
    # (build/abl/tpw1, same tree); the tx grid against HEAD~ (build/abl/r06prev)
    bash tools/gpu.sh $S tests || exit 1
    V="product tpw1"
    ABL_CFGS=c5 ABL_ARGS="$C5" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c4 ABL_ARGS="$C2" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    for v in new r06prev new r06prev new r06prev; do
      L=""; [ $v != new ] && L=build/abl/$v/libusn.so
      TAILN=1 TXB_ARGS="1048576 24 1 $L --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    ;;
  r06i)
    # tx: tile - 1's LAST/LREC and HEAD granules loaded ahead of the walk back
    # and the HEAD walk: tx tests, then the tx grid against HEAD~ (build/abl/r06prev)
    TESTS="tests/test_gpu_tx.py tests/test_gpu_parity.py" bash tools/gpu.sh $S tests || exit 1
    for v in new r06prev new r06prev new r06prev; do
      L=""; [ $v != new ] && L=build/abl/$v/libusn.so
      TAILN=1 TXB_ARGS="1048576 24 1 $L --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    ;;
  r06j)
    # the tree as it stands: the suite, smoke, the bench as the driver runs it,
    # rocprof of the bench, PMC of c5 / c2 and of the 8-ring tx call
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    bash tools/gpu.sh $S rocprof || exit 1
    PMC_CFGS="c5 c2" bash tools/gpu.sh $S pmc || exit 1
    TXB_ARGS="1048576 24 1 --rotate 8 --rings 8" bash tools/gpu.sh $S txprof txpmc || exit 1
    python3 tools/pmc_traffic.py gpurun_out/$S/txpmcf gpurun_out/$S/txpmcw 8388608 gpurun_out/$S/pmc_c4tx.json tx_kernel=1+33 > gpurun_out/$S/pmct_c4tx.log 2>&1
    ;;
  r06k)
    # tx: the probes' slot reads waited for after the records and the prefix
    # max (LDS-only barriers), keys recomputed from the records: tx and
    # parity tests, then the tx grid against HEAD~ (build/abl/r06prev)
    TESTS="tests/test_gpu_tx.py tests/test_gpu_parity.py tests/test_gpu_group.py tests/test_gpu_window.py" bash tools/gpu.sh $S tests || exit 1
    for v in new r06prev new r06prev new r06prev; do
      L=""; [ $v != new ] && L=build/abl/$v/libusn.so
      TAILN=1 TXB_ARGS="1048576 24 1 $L --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    ;;
  r06l)
    # r06k's A/B built r06prev from the same commit (identical ISA): the
    # order of the runs, not the code, measured?  reversed order plus a
    # byte copy of the product library at another path
    mkdir -p build/abl/copy && cp usnetd_amd/libusn.so build/abl/copy/libusn.so
    for v in r06prev new r06prev new copy new copy; do
      L=""; [ $v != new ] && L=build/abl/$v/libusn.so
      TAILN=1 TXB_ARGS="1048576 24 1 $L --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    ;;
  r06m)
    # wave priority A/Bs (s_setprio, USN_AB_TXPRIO / USN_AB_RXPRIO builds of
    # tools/abl_flags.sh; build/abl/base = the same flags-free build): the tx
    # grid per variant, twice; c5 / c2 classify calls interleaved in one process
    for v in base txp1 txp2 txp3 base txp1 txp2 txp3; do
      TAILN=1 TXB_ARGS="1048576 24 1 build/abl/$v/libusn.so --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    V="base rxp1 rxp2"
    ABL_CFGS=c5 ABL_ARGS="$C5" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c2 ABL_ARGS="$C2" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ;;
  r06n)
    # r06m's best tx variant (txp3: high priority while the header loads
    # issue) against base and two combinations, three times each
    for v in base txp3 txp4 txp5 base txp3 txp4 txp5 base txp3 txp4 txp5; do
      TAILN=1 TXB_ARGS="1048576 24 1 build/abl/$v/libusn.so --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    ;;
  r06o)
    # the tree with the tx wave priority (r06n): the suite, smoke, the bench
    # as the driver runs it, rocprof, PMC of c5 / c2 and of the 8-ring tx call
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    bash tools/gpu.sh $S rocprof || exit 1
    PMC_CFGS="c5 c2" bash tools/gpu.sh $S pmc || exit 1
    TXB_ARGS="1048576 24 1 --rotate 8 --rings 8" bash tools/gpu.sh $S txprof txpmc || exit 1
    python3 tools/pmc_traffic.py gpurun_out/$S/txpmcf gpurun_out/$S/txpmcw 8388608 gpurun_out/$S/pmc_c4tx.json tx_kernel=1+33 > gpurun_out/$S/pmct_c4tx.log 2>&1
    ;;
  r06p)
    # tx priority 6 (phase 2 at 2) and the scatter's load-issue priority
    # (USN_AB_SCPRIO) against base (= the product's priorities), tx grid
    # three times each; rx calls of c5 / c2 / c3 interleaved in one process
    for v in base txp6 scp1 base txp6 scp1 base txp6 scp1; do
      TAILN=1 TXB_ARGS="1048576 24 1 build/abl/$v/libusn.so --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    V="base scp1"
    ABL_CFGS=c5 ABL_ARGS="$C5" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c2 ABL_ARGS="$C2" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c3 ABL_ARGS="$C3" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ;;
  r06q)
    # tx: the LDS state zeroed after the header loads issue (no full barrier
    # ahead of them): tx and parity tests, then the tx grid against HEAD~
    # (build/abl/r06prev), alternating, the previous build first
    TESTS="tests/test_gpu_tx.py tests/test_gpu_parity.py tests/test_gpu_group.py tests/test_gpu_window.py" bash tools/gpu.sh $S tests || exit 1
    for v in r06prev new r06prev new r06prev new r06prev new; do
      L=""; [ $v != new ] && L=build/abl/$v/libusn.so
      TAILN=1 TXB_ARGS="1048576 24 1 $L --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    ;;
  r06r)
    # c4tx end to end: how much of the gap to the device rate is the timed
    # loop's fill and drain (13 launches by default) -- 13, 50 and 100 launches
    for L in 13 50 100 13 50 100; do
      BENCH_ARGS="--steps 10 --warmup 2 --no-cpu-baseline --extras c4tx --host-inclusive= --tx-launches $L" bash tools/gpu.sh $S bench || exit 1
      mv gpurun_out/$S/bench.log gpurun_out/$S/bench_tx${L}_$RANDOM.log
    done
    ;;
  r06s)
    # the tree with the early tx loads and the 50-launch c4tx loop: the
    # suite, smoke, the bench as the driver runs it, rocprof, PMC
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    bash tools/gpu.sh $S rocprof || exit 1
    PMC_CFGS="c5 c2" bash tools/gpu.sh $S pmc || exit 1
    TXB_ARGS="1048576 24 1 --rotate 8 --rings 8" bash tools/gpu.sh $S txprof txpmc || exit 1
    python3 tools/pmc_traffic.py gpurun_out/$S/txpmcf gpurun_out/$S/txpmcw 8388608 gpurun_out/$S/pmc_c4tx.json tx_kernel=1+33 > gpurun_out/$S/pmct_c4tx.log 2>&1
    ;;
  r06t)
    # the image's slot reads (one scattered 16-B read per frame) with an L1
    # bypass policy (USN_SLOT_POL: sc1, nt, sc0 sc1) against the default:
    # c5 / c4 / c3 classify calls interleaved in one process, twice
    V="base polsc1 polnt polsc01"
    ABL_CFGS=c5 ABL_ARGS="$C5" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c4 ABL_ARGS="$C2" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c3 ABL_ARGS="$C3" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    mv gpurun_out/$S/abl_c5.log gpurun_out/$S/abl_c5_1.log
    ABL_CFGS=c5 ABL_ARGS="$C5" ABL_VARIANTS="polnt polsc01 polsc1 base" bash tools/gpu.sh $S abl || exit 1
    # tx: the probes' displacement and slot reads as buffer loads with a
    # cache policy (USN_TX_AUX: 0 default, 2 nt, 16 sc1)
    for v in base txaux0 txaux2 txaux16 txaux16 txaux2 txaux0 base; do
      TAILN=1 TXB_ARGS="1048576 24 1 build/abl/$v/libusn.so --rotate 8 --rings 8" bash tools/gpu.sh $S txbench || exit 1
      mv gpurun_out/$S/txbench.log gpurun_out/$S/txbench_${v}_$RANDOM.log
    done
    ;;
  r06u)
    # DHCP requests from 0.0.0.0/8 sources other than 0.0.0.0 inside c4tx
    # rings (one ring, eight rings per grid) and DHCP-shaped frames from
    # outside 0/8, against the oracle
    TESTS="tests/test_gpu_tx.py" TEST_K="host_tail or not_unspecified" bash tools/gpu.sh $S tests || exit 1
    ;;
  r06v)
    # differential fuzz of the final tree (random streams with 0/8 DHCP
    # sources, sending runs split into 2-8 rings per launch) against the C
    # oracle: small images (LDS) and images past LDS (U and X probes)
    mkdir -p gpurun_out/$S
    for c in 0 1 2; do
      timeout -k 10 240 python -u tools/fuzz_multi_ring.py $((6000 + 100 * c)) 100 3000 > gpurun_out/$S/fuzz_$c.log 2>&1 \
        || { tail -3 gpurun_out/$S/fuzz_$c.log; exit 1; }
      tail -1 gpurun_out/$S/fuzz_$c.log
    done
    for c in 0 1; do
      timeout -k 10 240 python -u tools/fuzz_multi_ring.py $((7000 + 50 * c)) 50 3000 3000 > gpurun_out/$S/fuzzf_$c.log 2>&1 \
        || { tail -3 gpurun_out/$S/fuzzf_$c.log; exit 1; }
      tail -1 gpurun_out/$S/fuzzf_$c.log
    done
    ;;
  r06w)
    # the host-mapped state's device addresses cached per replica: the
    # suite, smoke, the bench as the driver runs it
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    ;;
  r06x)
    # the cached mapped-state addresses against HEAD~ (build/abl/r06prev),
    # interleaved in one process: c3 / c2 / c5 calls; then rocprof of the bench
    V="product r06prev"
    ABL_CFGS=c3 ABL_ARGS="$C3" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c2 ABL_ARGS="$C2" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c5 ABL_ARGS="$C5" ABL_VARIANTS="$V" bash tools/gpu.sh $S abl || exit 1
    bash tools/gpu.sh $S rocprof || exit 1
    ;;
  r06y)
    # host time of usn_classify_multi by checkpoint (test build, tools/hostprof.py)
    mkdir -p gpurun_out/$S
    for c in c3 c2 c5; do
      timeout -k 10 240 python -u tools/hostprof.py $c 400 > gpurun_out/$S/hostprof_$c.log 2>&1 || { tail -3 gpurun_out/$S/hostprof_$c.log; exit 1; }
      tail -1 gpurun_out/$S/hostprof_$c.log
    done
    ;;
  r06z)
    # the final tree's bench three times on one box (run-to-run spread)
    for k in 1 2 3; do
      BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
      mv gpurun_out/$S/bench.log gpurun_out/$S/bench_$k.log
    done
    ;;
  r06zz)
    # the final tree (test build with the host checkpoints): the suite and smoke
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    ;;
  *) echo "unknown session $S"; exit 2 ;;
esac
