#!/bin/bash
# Round-4 GPU sessions (each a sequence of tools/gpu.sh steps):
#   bash tools/r04.sh <session>   output under gpurun_out/<session>/
set -o pipefail
S=${1:?session}
O=gpurun_out/$S
mkdir -p $O
export TMPDIR=/tmp
case $S in
  r04a)
    # round-4 first session: the whole GPU suite (loud scatter errors, the
    # stale walk naming a new endpoint), smoke, the default bench (c1 keys,
    # c4tx at 100 rings), and the FETCH_SIZE calibration of one scattered
    # window read per 2048-byte slot (c3's pattern) from TCC_EA0_RDREQ
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
    for c in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" FETCH_SIZE; do
      n=$(echo $c | cut -d' ' -f1)
      rm -rf $O/sf_$n
      timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/sf_$n -o run -- build/stride_floor 4194304 2048 6 > $O/sf_$n.log 2>&1 || exit 1
    done
    ;;
  r04b)
    # tx lists built inside the tx launch (tx_lists): the GPU suite, tx ring
    # timing inline vs the scan + scatter launches, the scatter at 3 vs 2
    # workgroups per CU (80 vs 85 VGPRs), the default bench
    bash tools/gpu.sh $S testsall || exit 1
    TXB_ARGS="1048576 40 1 --rotate 6" bash tools/gpu.sh $S txbench || exit 1
    mv $O/txbench.log $O/txbench_inline.log
    USN_TX_LISTS_LAUNCHES=1 TXB_ARGS="1048576 40 1 --rotate 6" bash tools/gpu.sh $S txbench || exit 1
    mv $O/txbench.log $O/txbench_launches.log
    SCB_CFGS="c5 c2" SCB_VARIANTS="base scwpe4" bash tools/gpu.sh $S scb || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    TXB_ARGS="1048576 24 1 --rotate 6" bash tools/gpu.sh $S txprof
    ;;
  r04c)
    # tx inline lists with one polling wave per tile; rx inline removed (slower,
    # and two concurrent launches could each hold half the CUs); the suite,
    # tx ring timing inline vs launches, c3 PMC traffic with the x1 classify
    # fetch factor, the default bench
    bash tools/gpu.sh $S testsall || exit 1
    TXB_ARGS="1048576 40 1 --rotate 6" bash tools/gpu.sh $S txbench || exit 1
    mv $O/txbench.log $O/txbench_inline.log
    USN_TX_LISTS_LAUNCHES=1 TXB_ARGS="1048576 40 1 --rotate 6" bash tools/gpu.sh $S txbench || exit 1
    mv $O/txbench.log $O/txbench_launches.log
    TXB_ARGS="1048576 24 1 --rotate 6" bash tools/gpu.sh $S txprof || exit 1
    PMC_CFGS="c3" bash tools/gpu.sh $S pmc || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh $S bench
    ;;
  r04d)
    # tx rings pipelined (ring k + 1 before ring k's finalize): the suite, the
    # bench (c4tx pipelined + sequential), c3 PMC at the bench's launch shape
    bash tools/gpu.sh $S testsall || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    PMC_CFGS="c3" bash tools/gpu.sh $S pmc || exit 1
    SCB_CFGS="c5 c2" SCB_VARIANTS="base scnochk scwpe4" bash tools/gpu.sh $S scb
    ;;
  r04e)
    # final-tree counters and kernel breakdown: rocprof of the bench (per
    # kernel medians), PMC traffic of c5 / c2 / c4 and of the tx call
    bash tools/gpu.sh $S rocprof || exit 1
    PMC_CFGS="c5 c2 c4" bash tools/gpu.sh $S pmc || exit 1
    TXB_ARGS="1048576 24 1 --rotate 6" bash tools/gpu.sh $S txpmc || exit 1
    python3 tools/pmc_traffic.py $O/txpmcf $O/txpmcw 1048576 $O/pmc_c4tx.json > $O/pmct_c4tx.log 2>&1
    ;;
  r04f)
    # u8 count rows with per-tile exception rows: the suite, scan + scatter
    # A/B against r04b's u16 rows, the bench, the kernel breakdown
    bash tools/gpu.sh $S testsall || exit 1
    SCB_CFGS="c5 c2" SCB_VARIANTS="base" bash tools/gpu.sh $S scb || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    bash tools/gpu.sh $S rocprof || exit 1
    # small launches (1024 tiles: a tx ring, c3's calls): chunk length A/B
    for tc in 1 2 4; do
      for c in c4 c3; do
        if [ $c = c4 ]; then A="--frames 1048576 --multi 1"; else A="--frames 262144 --multi 4"; fi
        USN_SCATTER_TC=$tc timeout -k 10 300 python tools/scatter_bench.py --config $c $A --launches 100 \
          > $O/scb_small_${c}_tc$tc.log 2>&1 || exit 1
      done
      USN_SCATTER_TC=$tc timeout -k 10 300 python tools/txbench.py 1048576 40 1 --rotate 6 \
        > $O/txbench_tc$tc.log 2>&1 || exit 1
    done
    ;;
  r04g)
    # u8 rows + exception rows (HEAD) against u16 rows (f078668) in one
    # process (tools/abl_commit.sh builds both): whole calls, then the lists
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --batches 4 --multi 2 --rounds 5 --launches 40" ABL_VARIANTS="u8rows u16rows" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS="c4 c2" ABL_ARGS="--frames 1048576 --batches 16 --multi 8 --rounds 5 --launches 40" ABL_VARIANTS="u8rows u16rows" bash tools/gpu.sh $S abl || exit 1
    SCB_CFGS="c5 c2" SCB_VARIANTS="u8rows u16rows" bash tools/gpu.sh $S scb
    ;;
  r04h)
    # u8 rows, branch-free loads: the scatter tests, then r04g's A/B
    mkdir -p $O
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
      tests/test_gpu_scatter.py > $O/pytest_scatter.log 2>&1 || { tail -30 $O/pytest_scatter.log; exit 1; }
    tail -2 $O/pytest_scatter.log
    bash tools/r04.sh r04g
    ;;
  r04i)
    # tx lists on the side stream (USN_TX_LISTS_SIDE=1) against the caller's
    # stream: the tx tests with the knob, then c4tx end to end, alternated
    mkdir -p $O
    USN_TX_LISTS_SIDE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
      tests/test_gpu_tx.py > $O/pytest_tx_side.log 2>&1 || { tail -30 $O/pytest_tx_side.log; exit 1; }
    tail -2 $O/pytest_tx_side.log
    for rep in 1 2 3; do
      for side in 0 1; do
        USN_TX_LISTS_SIDE=$side timeout -k 10 300 python tools/txpipe.py > $O/txpipe_side${side}_$rep.log 2>&1 || exit 1
        echo "side=$side $(tail -1 $O/txpipe_side${side}_$rep.log)"
      done
    done
    ;;
  r04j)
    # chunk length of small scatter launches (the knob now taken as is):
    # lists alone (c4 1M, c3 4 x 256K) and c4tx end to end
    mkdir -p $O
    for tc in 0 1 2 4 8; do
      for c in c4 c3; do
        if [ $c = c4 ]; then A="--frames 1048576 --multi 1"; else A="--frames 262144 --multi 4"; fi
        USN_SCATTER_TC=$tc timeout -k 10 300 python tools/scatter_bench.py --config $c $A --launches 100 \
          > $O/scb_small_${c}_tc$tc.log 2>&1 || exit 1
        echo "tc=$tc $c $(tail -1 $O/scb_small_${c}_tc$tc.log)"
      done
      USN_SCATTER_TC=$tc timeout -k 10 300 python tools/txpipe.py > $O/txpipe_tc$tc.log 2>&1 || exit 1
      echo "tc=$tc c4tx $(tail -1 $O/txpipe_tc$tc.log)"
    done
    ;;
  r04k)
    # one chunk per CU for small scatter launches: the suite and the bench
    bash tools/gpu.sh $S testsall || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh $S bench
    ;;
  r04l)
    # both rounds' header DMA at the workgroup start (USN_EARLY_R1, 3
    # workgroups per CU at c5's LDS) against the current build
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --batches 4 --multi 2 --rounds 5 --launches 40" ABL_VARIANTS="cur early1" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS="c4" ABL_ARGS="--frames 1048576 --batches 16 --multi 8 --rounds 5 --launches 40" ABL_VARIANTS="cur early1" bash tools/gpu.sh $S abl
    ;;
  r04m)
    # c3's lane path: bytes 12..43 in two loads (cur) against 0..47 in three
    ABL_CFGS=c3 ABL_ARGS="--frames 262144 --batches 16 --multi 4 --rounds 5 --launches 40" ABL_VARIANTS="cur lane48" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c3 ABL_ARGS="--frames 1048576 --batches 8 --multi 1 --rounds 5 --launches 40" ABL_VARIANTS="cur lane48" bash tools/gpu.sh $S abl
    ;;
  r04n)
    # small launches sum their count rows in the scatter (no scan launch):
    # the scatter tests, then USN_SELFSCAN_KB 0 (off) / 256 / 1024 on the lists
    # of c3's calls and a 1M c4 ring, and c4tx end to end
    mkdir -p $O
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
      tests/test_gpu_scatter.py tests/test_gpu_tx.py > $O/pytest_sel.log 2>&1 || { tail -30 $O/pytest_sel.log; exit 1; }
    tail -2 $O/pytest_sel.log
    for kb in 0 256 1024; do
      for c in c4 c3; do
        if [ $c = c4 ]; then A="--frames 1048576 --multi 1"; else A="--frames 262144 --multi 4"; fi
        USN_SELFSCAN_KB=$kb timeout -k 10 300 python tools/scatter_bench.py --config $c $A --launches 100 \
          > $O/scb_small_${c}_kb$kb.log 2>&1 || exit 1
        echo "kb=$kb $c $(tail -1 $O/scb_small_${c}_kb$kb.log)"
      done
      USN_SELFSCAN_KB=$kb timeout -k 10 300 python tools/txpipe.py > $O/txpipe_kb$kb.log 2>&1 || exit 1
      echo "kb=$kb c4tx $(tail -1 $O/txpipe_kb$kb.log)"
    done
    ;;
  r04o)
    # self-scan by bytes read: the suite and the bench
    bash tools/gpu.sh $S testsall || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh $S bench
    ;;
  r04p)
    # c3 under its bench key, self-scan off / on, alternated
    mkdir -p $O
    for rep in 1 2 3; do
      for kb in 0 16384; do
        USN_SELFSCAN_KB=$kb timeout -k 10 300 python bench.py --config c3 --queues 8 --no-extra --no-cpu-baseline \
          --steps 200 --warmup 20 > $O/c3_kb${kb}_$rep.log 2>&1 || exit 1
        echo "kb=$kb $(python3 tools/bench_summary.py $O/c3_kb${kb}_$rep.log | head -1)"
      done
    done
    ;;
  r04q)
    # self-scan with 16-byte row loads (registers instead of occupancy): the
    # scatter tests, c3 lists and bench key alternated with the scan, c3 PMC
    mkdir -p $O
    timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
      tests/test_gpu_scatter.py > $O/pytest_sel.log 2>&1 || { tail -30 $O/pytest_sel.log; exit 1; }
    tail -2 $O/pytest_sel.log
    for kb in 0 16384; do
      USN_SELFSCAN_KB=$kb timeout -k 10 300 python tools/scatter_bench.py --config c3 --frames 262144 --multi 4 \
        --launches 100 > $O/scb_c3_kb$kb.log 2>&1 || exit 1
      echo "kb=$kb c3 $(tail -1 $O/scb_c3_kb$kb.log)"
    done
    for rep in 1 2; do
      for kb in 0 16384; do
        USN_SELFSCAN_KB=$kb timeout -k 10 300 python bench.py --config c3 --queues 8 --no-extra --no-cpu-baseline \
          --steps 200 --warmup 20 > $O/c3_kb${kb}_$rep.log 2>&1 || exit 1
        echo "kb=$kb $(python3 tools/bench_summary.py $O/c3_kb${kb}_$rep.log | head -1)"
      done
    done
    PMC_CFGS="c3" bash tools/gpu.sh $S pmc
    ;;
  r04r)
    # the scatter tests (scan or self-scan), then nt decision reads in the
    # scatter (index runs' partial lines merging in L2) against the current
    mkdir -p $O
    timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
      tests/test_gpu_scatter.py > $O/pytest_scatter.log 2>&1 || { tail -30 $O/pytest_scatter.log; exit 1; }
    tail -2 $O/pytest_scatter.log
    SCB_CFGS="c5 c2" SCB_VARIANTS="cur scnt" bash tools/gpu.sh $S scb
    ;;
  r04s)
    # phase stamps of the tx kernel and the c5 classify (diagnostic build)
    STAMP_ARGS="c4tx 1048576" bash tools/gpu.sh $S stamps || exit 1
    mv $O/stamps.log $O/stamps_c4tx.log
    STAMP_ARGS="c5 8388608" bash tools/gpu.sh $S stamps
    mv $O/stamps.log $O/stamps_c5.log
    ;;
  r04t)
    # persistent classify (resident workgroups loop over tiles; 64 VGPRs, 36 B
    # spilled) against one workgroup per tile, c5 and c4
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --batches 4 --multi 2 --rounds 5 --launches 40" ABL_VARIANTS="cur persist" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS="c4 c2" ABL_ARGS="--frames 1048576 --batches 16 --multi 8 --rounds 5 --launches 40" ABL_VARIANTS="cur persist" bash tools/gpu.sh $S abl
    ;;
  r04z)
    # final tree: the suite, smoke, the bench as the driver runs it, rocprof
    # of the bench, PMC of c5 / c2 / c4 and of the tx call (mixed requests)
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    bash tools/gpu.sh $S rocprof || exit 1
    PMC_CFGS="c5 c2 c4" bash tools/gpu.sh $S pmc || exit 1
    TXB_ARGS="1048576 24 1 --rotate 6" bash tools/gpu.sh $S txpmc || exit 1
    python3 tools/pmc_traffic.py $O/txpmcf $O/txpmcw 1048576 $O/pmc_c4tx.json tx_kernel=1+32 > $O/pmct_c4tx.log 2>&1
    ;;
  r04u)
    # the scatter at 8 waves per SIMD (64 VGPRs, spills): c2's and c4's 1024
    # chunks in one generation of 4 workgroups per CU
    SCB_CFGS="c2 c4 c5" SCB_VARIANTS="cur scwpe8" bash tools/gpu.sh $S scb
    ;;
  r04v)
    # tx: records and prefix max under the rule probes' slot reads (txepfx,
    # since reverted) against the current, alternated, device time per ring
    mkdir -p $O
    for rep in 1 2 3; do
      for v in cur txepfx; do
        timeout -k 10 300 python tools/txbench.py 1048576 40 1 build/abl/$v/libusn.so --rotate 6 \
          > $O/txbench_${v}_$rep.log 2>&1 || exit 1
        echo "$v $(tail -1 $O/txbench_${v}_$rep.log | cut -c1-200)"
      done
    done
    ;;
  r04w)
    # self-scan past one generation (USN_SELFSCAN_ANY=1): c2's 8 x 1M call
    # (1024 chunks, 49 MB of rows read) with the row limit raised
    mkdir -p $O
    for rep in 1 2; do
      for v in "0 16384" "1 65536"; do
        set -- $v
        USN_SELFSCAN_ANY=$1 USN_SELFSCAN_KB=$2 timeout -k 10 300 python tools/scatter_bench.py --config c2 \
          --frames 1048576 --multi 8 --launches 100 > $O/scb_c2_any$1_$rep.log 2>&1 || exit 1
        echo "any=$1 kb=$2 $(tail -1 $O/scb_c2_any$1_$rep.log)"
      done
    done
    ;;
  r04x)
    # the PCIe-inclusive loop on the final tree (hostio.py), c2 and c5
    HOSTIO_ARGS="c2 1048576 8 4 6" bash tools/gpu.sh $S hostio || exit 1
    mv $O/hostio.log $O/hostio_c2.log
    HOSTIO_ARGS="c5 1048576 8 4 6" bash tools/gpu.sh $S hostio || exit 1
    mv $O/hostio.log $O/hostio_c5.log
    ;;
  r04y)
    # c2's PCIe-inclusive loop (1M rings on 4 streams): self-scan / scan /
    # the old 1-tile chunks
    mkdir -p $O
    for v in "16384 0" "0 0" "0 1"; do
      set -- $v
      USN_SELFSCAN_KB=$1 USN_SCATTER_TC=$2 timeout -k 10 300 python tools/hostio.py c2 1048576 8 4 6 \
        > $O/hostio_c2_kb$1_tc$2.log 2>&1 || exit 1
      echo "kb=$1 tc=$2 $(head -c 160 $O/hostio_c2_kb$1_tc$2.log)"
    done
    ;;
  r04aa)
    # the scatter_plan refactor and the earlier self-scan zeroing: scatter +
    # tx tests, then c3's lists against the previous commit, alternated
    mkdir -p $O
    timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
      tests/test_gpu_scatter.py tests/test_gpu_tx.py > $O/pytest_sel.log 2>&1 || { tail -30 $O/pytest_sel.log; exit 1; }
    tail -2 $O/pytest_sel.log
    for rep in 1 2; do
      timeout -k 10 300 python tools/scatter_bench.py --config c3 --frames 262144 --multi 4 --launches 100 \
        cur selfold > $O/scb_c3_$rep.log 2>&1 || exit 1
      grep scatter $O/scb_c3_$rep.log
    done
    ;;
  r04ab)
    # c3 with self-scan at 8-tile chunks (128 chunks) against the plan's 4
    mkdir -p $O
    for rep in 1 2; do
      for tc in 0 8; do
        USN_SCATTER_TC=$tc timeout -k 10 300 python tools/scatter_bench.py --config c3 --frames 262144 --multi 4 \
          --launches 100 > $O/scb_c3_tc${tc}_$rep.log 2>&1 || exit 1
        echo "tc=$tc $(grep scatter $O/scb_c3_tc${tc}_$rep.log)"
      done
    done
    ;;
  r04ac)
    # the scan inside the scatter for one resident batch (USN_SCF_FUSED, two
    # grid barriers; since reverted): the suite, then fused / scan on a tx
    # ring and 1M rings
    bash tools/gpu.sh $S testsall || exit 1
    for rep in 1 2; do
      for f in 0 1; do
        USN_FUSED=$f timeout -k 10 300 python tools/txpipe.py > $O/txpipe_f${f}_$rep.log 2>&1 || exit 1
        echo "fused=$f c4tx $(tail -1 $O/txpipe_f${f}_$rep.log)"
        for c in c4 c5; do
          USN_FUSED=$f timeout -k 10 300 python tools/scatter_bench.py --config $c --frames 1048576 --multi 1 \
            --launches 100 > $O/scb_${c}_f${f}_$rep.log 2>&1 || exit 1
          echo "fused=$f $c $(grep scatter $O/scb_${c}_f${f}_$rep.log)"
        done
      done
    done
    ;;
  r04ad)
    # the final tree again (after the reverted experiments): the suite, smoke,
    # the bench with the driver's defaults, rocprof of the bench
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    bash tools/gpu.sh $S rocprof
    ;;
  r04ae)
    # the classify's first barrier LDS-only (each wave waits for its own
    # round 0) against the current, c5 / c4 / c2
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --batches 4 --multi 2 --rounds 5 --launches 40" ABL_VARIANTS="cur bar0" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS="c4 c2" ABL_ARGS="--frames 1048576 --batches 16 --multi 8 --rounds 5 --launches 40" ABL_VARIANTS="cur bar0" bash tools/gpu.sh $S abl
    ;;
  r04af)
    # L2 hits and misses of the c5 call per kernel (are the U slot reads L2 hits?)
    mkdir -p $O
    rm -rf $O/l2
    timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/l2 -o run -- \
      python3 bench.py --config c5 --no-extra --steps 16 --warmup 4 --no-cpu-baseline --launch-probe 0 --ramp 0 \
      > $O/l2.log 2>&1 || exit 1
    python3 - $O/l2 <<'PY'
import csv, glob, os, sys
from collections import defaultdict
tot = defaultdict(float); n = defaultdict(int)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        if r["Counter_Name"] == "TCC_HIT_sum": n[k] += 1
for (k, c), v in sorted(tot.items()):
    print("%-42s %-14s %14.0f per dispatch %12.0f" % (k, c, v, v / max(1, n[k])))
PY
    ;;
  r04ag)
    # wave priority for the classify tile's tail (prio2) against the current
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --batches 4 --multi 2 --rounds 5 --launches 40" ABL_VARIANTS="cur prio2" bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS="c4 c2" ABL_ARGS="--frames 1048576 --batches 16 --multi 8 --rounds 5 --launches 40" ABL_VARIANTS="cur prio2" bash tools/gpu.sh $S abl
    ;;
  r04ah)
    # the driver's multi-GPU launch shape rehearsed on one GPU (two ranks)
    bash tools/gpu.sh $S bench_n2
    ;;
  r04ai)
    # c4tx timed without events in the pipelined loop (events in a second pass)
    mkdir -p $O
    for rep in 1 2 3; do
      timeout -k 10 300 python tools/txpipe.py > $O/txpipe_$rep.log 2>&1 || exit 1
      tail -1 $O/txpipe_$rep.log
    done
    ;;
  r04aj)
    # the bench line with c4tx timed without events in its loop
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench
    ;;
  *) echo "unknown session $S"; exit 2 ;;
esac
echo "== session $S done"
