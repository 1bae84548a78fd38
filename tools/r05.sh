#!/bin/bash
# Round-5 GPU sessions (each a sequence of tools/gpu.sh steps):
#   bash tools/r05.sh <session>   output under gpurun_out/<session>/
set -o pipefail
S=${1:?session}
O=gpurun_out/$S
mkdir -p $O
export TMPDIR=/tmp
sq_pass() {   # sq_pass NAME "COUNTERS" CMD...: one rocprofv3 --pmc pass (<= 8 SQ counters)
  local name=$1 ctr=$2; shift 2
  rm -rf $O/$name
  timeout -k 10 180 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$name -o run -- "$@" \
    > $O/$name.log 2>&1 || { echo "pmc pass $name failed rc=$?"; exit 1; }
}
case $S in
  r05a)
    # first session of the round: the whole GPU suite (with the headline
    # launch's parity test), smoke, the driver's bench, and the c5
    # classify's instruction mix and wave cycles (SQ counters, two passes)
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
    sq_pass sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
      python3 tools/kbench.py c5 8388608 12
    sq_pass sq2 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
      python3 tools/kbench.py c5 8388608 12
    python3 tools/pmc_summary.py $O/sq1 $O/sq2 > $O/sq_summary.txt 2>&1 || true
    ;;
  r05b)
    # classify_chunk_kernel (pipelined wave-per-tile classify, one count row
    # per chunk) + the self-counting scatter: the GPU suite, A/B against the
    # one-tile-per-workgroup classify in one process (c5 2 x 8M, c4 8 x 1M),
    # the driver's bench
    bash tools/gpu.sh $S testsall || exit 1
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --multi 2 --rounds 5 --launches 40" ABL_VARIANTS="base nochunk" \
      bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c4 ABL_ARGS="--frames 1048576 --multi 8 --rounds 5 --launches 40" ABL_VARIANTS="base nochunk" \
      bash tools/gpu.sh $S abl || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    ;;
  r05c)
    # where the chunk kernel's call time goes: rocprof kernel stats of the
    # A/B (base: classify_chunk_kernel + chunk-row scan + counting scatter;
    # nochunk: round 4's three kernels), c5 2 x 8M and c4 8 x 1M
    rm -rf $O/prof5 $O/prof4
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof5 -o run -- \
      python3 tools/abl.py --config c5 --frames 8388608 --multi 2 --batches 4 --rounds 3 --launches 30 \
      --json $O/abl_c5.json base nochunk > $O/abl_c5.log 2>&1 || exit 1
    python3 tools/trace_summary.py $O/prof5/run_kernel_trace.csv > $O/trace_c5.log 2>&1
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4 -o run -- \
      python3 tools/abl.py --config c4 --frames 1048576 --multi 8 --batches 8 --rounds 3 --launches 30 \
      --json $O/abl_c4.json base nochunk > $O/abl_c4.log 2>&1 || exit 1
    python3 tools/trace_summary.py $O/prof4/run_kernel_trace.csv > $O/trace_c4.log 2>&1
    ;;
  r05d)
    # instruction mix of classify_chunk_kernel against classify_rx_kernel
    # (SQ counters, two passes over the A/B harness, c5 2 x 8M)
    A="tools/abl.py --config c5 --frames 8388608 --multi 2 --batches 4 --rounds 1 --launches 6 base nochunk"
    sq_pass sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" python3 $A
    sq_pass sq2 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU" python3 $A
    python3 tools/pmc_summary.py $O/sq1 $O/sq2 > $O/sq_summary.txt 2>&1 || true
    ;;
  r05e)
    # classify_chunk_kernel variants (steady steps as a loop over pairs at 64
    # VGPRs, the same at 80, the 16-step unroll) against round 4's classify:
    # rocprof kernel stats of the A/B harness, c5 2 x 8M and c4 8 x 1M; then the
    # volume parity tests on the default build
    for c in c5 c4; do
      if [ $c = c5 ]; then A="--frames 8388608 --multi 2 --batches 4"; else A="--frames 1048576 --multi 8 --batches 8"; fi
      rm -rf $O/prof_$c
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- \
        python3 tools/abl.py --config $c $A --rounds 3 --launches 30 --json $O/abl_$c.json \
        base ckloop ckwpe6 nochunk > $O/abl_$c.log 2>&1 || exit 1
      python3 tools/trace_summary.py $O/prof_$c/run_kernel_trace.csv > $O/trace_$c.log 2>&1
    done
    bash tools/gpu.sh $S testsall || exit 1
    BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    ;;
  r05f)
    # A/B: the chunk kernel with interleaved segments (a workgroup's waves
    # read 512 consecutive frames at a time) against its tile-per-wave order
    # and round 4's classify
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --multi 2 --batches 4 --rounds 5 --launches 30" ABL_VARIANTS="base ckinter nochunk" \
      bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c4 ABL_ARGS="--frames 1048576 --multi 8 --batches 8 --rounds 5 --launches 30" ABL_VARIANTS="base ckinter nochunk" \
      bash tools/gpu.sh $S abl || exit 1
    ;;
  r05g)
    # two consecutive rings per tx launch (one grid): the tx GPU tests, the
    # bench's c4tx line (one ring per launch and two, pipelined)
    TESTS=tests/test_gpu_tx.py bash tools/gpu.sh $S testsall || exit 1
    BENCH_ARGS="--steps 10 --warmup 3 --extras c4tx --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    ;;
  r05h)
    # two rings per tx launch, round 2: the tx GPU tests, the c4tx line, the
    # kernel times and HBM traffic of a two-ring launch (6 rotating buffers)
    TESTS=tests/test_gpu_tx.py bash tools/gpu.sh $S testsall || exit 1
    BENCH_ARGS="--steps 10 --warmup 3 --extras c4tx --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    TXB_ARGS="1048576 24 1 --rotate 6 --rings 2" bash tools/gpu.sh $S txprof txpmc || exit 1
    python3 tools/pmc_traffic.py $O/txpmcf $O/txpmcw 2097152 $O/pmc_c4tx2.json tx_kernel=1+32 > $O/pmct_c4tx2.log 2>&1
    ;;
  r05i)
    # the tx PMC model's calibration: TCC request counters
    # of tools/tx_pmc_cal.hip's kernels (one request type each, known units)
    # and of a two-ring tx call, three passes each
    TX="tools/txbench.py 1048576 12 1 --rotate 6 --rings 2"
    P1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum"
    P2="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
    timeout -k 10 120 build/tx_pmc_cal > $O/cal_time.log 2>&1 || exit 1
    sq_pass calr "$P1" build/tx_pmc_cal
    sq_pass calw "$P2" build/tx_pmc_cal
    sq_pass calf FETCH_SIZE build/tx_pmc_cal
    sq_pass txr "$P1" python3 $TX
    sq_pass txw "$P2" python3 $TX
    sq_pass txf FETCH_SIZE python3 $TX
    python3 tools/pmc_cal_summary.py 2097152 $O/pmc_cal.json $O/calr $O/calw $O/calf $O/txr $O/txw $O/txf > $O/pmc_cal.log 2>&1
    ;;
  r05j)
    # the scatter deriving its per-tile counts from the decisions in LDS (no
    # count-row reads; the scan's sums checked against them) against the
    # row-reading scatter (HEAD, build/abl/scrows): scatter tests, scan +
    # scatter device time, whole calls
    TESTS="tests/test_gpu_scatter.py tests/test_gpu_volume.py" bash tools/gpu.sh $S testsall || exit 1
    SCB_CFGS="c5 c2 c4" SCB_VARIANTS="base scrows" bash tools/gpu.sh $S scb || exit 1
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --multi 2 --batches 4 --rounds 5 --launches 30" ABL_VARIANTS="base scrows" \
      bash tools/gpu.sh $S abl || exit 1
    ;;
  r05k)
    # the ADVICE r04 regression tests (the host tail's carried cache across a
    # refused finalize; a tx finalize on another stream) with the tx suite
    TESTS="tests/test_gpu_window.py tests/test_gpu_tx.py" bash tools/gpu.sh $S testsall || exit 1
    ;;
  r05z)
    # final tree: the suite, smoke, the bench as the driver runs it, rocprof
    # of the bench, PMC of c5 / c2 / c3 / c4 and of the two-ring tx call
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    bash tools/gpu.sh $S rocprof || exit 1
    PMC_CFGS="c5 c2 c3 c4" bash tools/gpu.sh $S pmc || exit 1
    TXB_ARGS="1048576 24 1 --rotate 6 --rings 2" bash tools/gpu.sh $S txprof txpmc || exit 1
    python3 tools/pmc_traffic.py $O/txpmcf $O/txpmcw 2097152 $O/pmc_c4tx.json tx_kernel=1+33 > $O/pmct_c4tx.log 2>&1
    ;;
  r05l)
    # the bench's end-to-end loops with their ctypes arguments built once
    BENCH_ARGS="--steps 20 --warmup 3 --extras c2,c3,c4tx --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    ;;
  r05m)
    # an rx usn_finalize waits for its own launch's event, not the stream:
    # the suite, then the end-to-end loops
    bash tools/gpu.sh $S testsall || exit 1
    BENCH_ARGS="--steps 20 --warmup 3 --extras c2,c3,c4 --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    ;;
  r05n)
    # the two-ring tile-edge tests; the end-to-end loops' steady state
    TESTS=tests/test_gpu_tx.py TEST_K=tile_edges bash tools/gpu.sh $S testsall || exit 1
    BENCH_ARGS="--steps 40 --warmup 5 --extras c3 --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    ;;
  r05o)
    # where the end-to-end loop's host time goes (c3, c2, c5)
    for c in c3 c2 c5; do
      timeout -k 10 240 python3 tools/e2e_trace.py $c 200 > $O/e2e_$c.log 2>&1 || exit 1
    done
    ;;
  r05p)
    # results double-buffered in the bench: the end-to-end loop's host time,
    # then the bench line
    for c in c3 c2 c5; do
      timeout -k 10 240 python3 tools/e2e_trace.py $c 200 > $O/e2e_$c.log 2>&1 || exit 1
    done
    BENCH_ARGS="--steps 40 --warmup 5 --extras c2,c3,c4 --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    TESTS=tests/test_gpu_bench.py bash tools/gpu.sh $S testsall || exit 1
    ;;
  r05q)
    # A/B in turn on one box: result buffers of one round against two (the
    # value loop's outputs stay MALL-resident when every round rewrites the same)
    for rr in 1 2 1 2; do
      timeout -k 10 300 python bench.py --steps 40 --warmup 5 --extras c2,c3 --no-cpu-baseline \
        --result-rounds $rr > $O/bench_rr$rr.log 2>&1 || exit 1
      python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench_rr$rr.log') if l.startswith('{')][-1]); print('rr=$rr', d['value'], d['end_to_end_mpps'], d['c2']['value'], d['c3']['value'])"
    done
    ;;
  r05r)
    # the value loop on one round's results, the end-to-end loop on two
    BENCH_ARGS="--steps 40 --warmup 5 --extras c2,c3,c4 --no-cpu-baseline" bash tools/gpu.sh $S bench || exit 1
    TESTS=tests/test_gpu_bench.py bash tools/gpu.sh $S testsall || exit 1
    ;;
  r05s)
    # the c5 scan's chunks per thread (product: 4, 512 workgroups) against 2
    # and 1 (the test build's USN_SCAN_CPT knob), scan + scatter device time
    for cpt in 2 1; do
      USN_SCAN_CPT=$cpt timeout -k 10 300 python tools/scatter_bench.py --config c5 --frames 8388608 --multi 2 \
        --json $O/scb_cpt$cpt.json base testlib > $O/scb_cpt$cpt.log 2>&1 || exit 1
      cat $O/scb_cpt$cpt.log | grep scatter
    done
    ;;
  r05t)
    # the scan with 16-byte row loads (scan16_kernel) against 8-byte
    # (build/abl/scan8 = HEAD): the lists' tests, scan + scatter device time
    TESTS="tests/test_gpu_scatter.py tests/test_gpu_volume.py" bash tools/gpu.sh $S testsall || exit 1
    SCB_CFGS="c5 c2 c4" SCB_VARIANTS="base scan8 base scan8" bash tools/gpu.sh $S scb || exit 1
    ;;
  r05y)
    # final tree (after the rx finalize event and the bench's result
    # buffering): the suite, smoke, the bench as the driver runs it, rocprof
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    bash tools/gpu.sh $S rocprof || exit 1
    ;;
  r05u)
    # what the rx launch's completion event costs: the product library against
    # the commit before it (build/abl/noev), whole calls in the bench's shapes
    ABL_CFGS=c3 ABL_ARGS="--frames 262144 --multi 4 --batches 16 --streams 2 --rounds 5 --launches 60" ABL_VARIANTS="base noev" \
      bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c2 ABL_ARGS="--frames 1048576 --multi 8 --batches 16 --streams 2 --rounds 5 --launches 40" ABL_VARIANTS="base noev" \
      bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --multi 2 --batches 4 --rounds 5 --launches 30" ABL_VARIANTS="base noev" \
      bash tools/gpu.sh $S abl || exit 1
    ;;
  r05v)
    # the rx completion event's flags: default (system fence), device-scope
    # release, no system fence, against no event (build/abl/noev), c5 and c2
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --multi 2 --batches 4 --rounds 5 --launches 30" ABL_VARIANTS="base noev evdev evnofence" \
      bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c4 ABL_ARGS="--frames 1048576 --multi 8 --batches 16 --rounds 5 --launches 40" ABL_VARIANTS="base noev evdev evnofence" \
      bash tools/gpu.sh $S abl || exit 1
    ;;
  r05w)
    # completion events without the system fence (rx and tx): the suite,
    # smoke, the A/B against the fenced events (build/abl/sysfence), the
    # c4tx pipeline (txpipe), the bench
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --multi 2 --batches 4 --rounds 5 --launches 30" ABL_VARIANTS="base sysfence noev" \
      bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c4 ABL_ARGS="--frames 1048576 --multi 8 --batches 16 --rounds 5 --launches 40" ABL_VARIANTS="base sysfence noev" \
      bash tools/gpu.sh $S abl || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    ;;
  r05x)
    # the classify's header stage at the two parts it loads (16 KiB: c5 at 4
    # workgroups per CU) against 3 parts (build/abl/stage192 = HEAD)
    TESTS="tests/test_gpu_volume.py tests/test_gpu_parity.py" bash tools/gpu.sh $S testsall || exit 1
    ABL_CFGS=c5 ABL_ARGS="--frames 8388608 --multi 2 --batches 4 --rounds 8 --launches 30" ABL_VARIANTS="product stage192" \
      bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS="c4 c2" ABL_ARGS="--frames 1048576 --multi 8 --batches 16 --rounds 5 --launches 40" ABL_VARIANTS="product stage192" \
      bash tools/gpu.sh $S abl || exit 1
    ABL_CFGS=c3 ABL_ARGS="--frames 262144 --multi 4 --batches 16 --streams 2 --rounds 5 --launches 60" ABL_VARIANTS="product stage192" \
      bash tools/gpu.sh $S abl || exit 1
    ;;
  r05aa)
    # a two-ring tx grid handing its carried cache to another replica
    TESTS="tests/test_gpu_group.py tests/test_gpu_tx.py" bash tools/gpu.sh $S testsall || exit 1
    ;;
  r05ab)
    # flake check: the whole GPU suite twice, then smoke
    TAILN=3 bash tools/gpu.sh $S testsall || exit 1
    mv $O/pytest_gpu.log $O/pytest_gpu_1.log
    TAILN=3 bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    ;;
  r05ac)
    # the scatter ranking few-bin launches by bit-sliced match (one atomic per
    # distinct bin of a segment; c2's 19 bins) against atomics per frame
    # (build/abl/scold = HEAD), and with the threshold at 2^7 bins (c3's 69)
    TESTS="tests/test_gpu_scatter.py tests/test_gpu_parity.py" bash tools/gpu.sh $S testsall || exit 1
    SCB_CFGS="c2 c5" SCB_VARIANTS="base scold scmatch7" bash tools/gpu.sh $S scb || exit 1
    for c in c3 c1; do
      timeout -k 10 300 python tools/scatter_bench.py --config $c --frames 262144 --multi 4 \
        --json $O/scb_$c.json base scold scmatch7 > $O/scb_$c.log 2>&1 || exit 1
      grep scatter $O/scb_$c.log
    done
    ;;
  r05ad)
    # the scatter's chunk length for c2 / c4 (8 x 1M per call; product: 8
    # tiles, 1024 chunks in one generation) at 4 and 2 (the test build's
    # USN_SCATTER_TC knob)
    for tc in 4 2; do
      for c in c2 c4; do
        USN_SCATTER_TC=$tc timeout -k 10 300 python tools/scatter_bench.py --config $c --frames 1048576 --multi 8 \
          base testlib > $O/scb_${c}_tc$tc.log 2>&1 || exit 1
        echo "tc=$tc $c"; grep scatter $O/scb_${c}_tc$tc.log
      done
    done
    ;;
  r05ae)
    # a two-ring tx launch's lists at 4-tile chunks (512 chunks: two per CU)
    # against the plan's 8 (256, one per CU): the test build's USN_SCATTER_TC
    for rep in 1 2; do
      timeout -k 10 200 python tools/txbench.py 1048576 24 1 --rotate 6 --rings 2 > $O/txb_prod_$rep.log 2>&1 || exit 1
      USN_SCATTER_TC=4 timeout -k 10 200 python tools/txbench.py 1048576 24 1 build/test/libusn.so --rotate 6 --rings 2 \
        > $O/txb_tc4_$rep.log 2>&1 || exit 1
      tail -1 $O/txb_prod_$rep.log; tail -1 $O/txb_tc4_$rep.log
    done
    ;;
  r05af)
    # the new two-ring random-stream parity tests, then a differential fuzz
    # of two-ring tx launches (tools/fuzz_two_ring.py, since renamed
    # fuzz_multi_ring.py and splitting into 2-4 rings; 200 seeds in 4 chunks)
    TESTS="tests/test_gpu_parity.py" bash tools/gpu.sh $S testsall || exit 1
    for c in 0 1 2 3; do
      timeout -k 10 240 python -u tools/fuzz_multi_ring.py $((1000 + 50 * c)) 50 3000 > $O/fuzz_$c.log 2>&1 \
        || { tail -3 $O/fuzz_$c.log; exit 1; }
      tail -1 $O/fuzz_$c.log
    done
    ;;
  r05ag)
    # per-frame tx cost against the grid's size, same flows (--concat: a ring
    # of K copies of the 1M c4tx ring): 1M x 2 rings (the product's launch),
    # 2M x 1, 2M x 2 (a 4M grid, as four 1M rings would be), 4M x 1
    for rep in 1 2; do
      timeout -k 10 200 python tools/txbench.py 1048576 24 1 --rotate 6 --rings 2 > $O/txb_1Mx2_$rep.log 2>&1 || exit 1
      timeout -k 10 200 python tools/txbench.py 1048576 24 1 --rotate 3 --concat 2 --rings 1 > $O/txb_2Mx1_$rep.log 2>&1 || exit 1
      timeout -k 10 200 python tools/txbench.py 1048576 24 1 --rotate 3 --concat 2 --rings 2 > $O/txb_2Mx2_$rep.log 2>&1 || exit 1
      timeout -k 10 200 python tools/txbench.py 1048576 24 1 --rotate 2 --concat 4 --rings 1 > $O/txb_4Mx1_$rep.log 2>&1 || exit 1
      for v in 1Mx2 2Mx1 2Mx2 4Mx1; do echo "$v $(tail -1 $O/txb_${v}_$rep.log)"; done
    done
    ;;
  r05ah)
    # up to four consecutive rings per tx launch (one grid): the tx and
    # random-stream GPU tests, a multi-ring fuzz, 2 vs 4 rings per launch
    # (txbench, 8 rotating buffers), the bench's c4tx line at 2 and 4
    TESTS="tests/test_gpu_tx.py tests/test_gpu_parity.py tests/test_gpu_window.py tests/test_gpu_group.py" \
      bash tools/gpu.sh $S testsall || exit 1
    timeout -k 10 240 python -u tools/fuzz_multi_ring.py 2000 100 3000 > $O/fuzz.log 2>&1 || { tail -3 $O/fuzz.log; exit 1; }
    tail -1 $O/fuzz.log
    for rep in 1 2; do
      for r in 2 4; do
        timeout -k 10 200 python tools/txbench.py 1048576 24 1 --rotate 8 --rings $r > $O/txb_r${r}_$rep.log 2>&1 || exit 1
        echo "rings=$r $(tail -1 $O/txb_r${r}_$rep.log)"
      done
    done
    for r in 2 4; do
      BENCH_ARGS="--steps 10 --warmup 3 --extras c4tx --no-cpu-baseline --tx-rings $r" bash tools/gpu.sh $S bench || exit 1
      mv $O/bench.log $O/bench_tx$r.log
    done
    ;;
  r05ai)
    # four-ring tx launches: kernel times (rocprof) and HBM traffic of one
    # launch (8 rotating buffers), for the bench line's roofline; an 8M grid
    # (4 rings of 2M, --concat 2: the same flows) against 4 x 1M
    TXB_ARGS="1048576 24 1 --rotate 8 --rings 4" bash tools/gpu.sh $S txprof txpmc || exit 1
    python3 tools/pmc_traffic.py $O/txpmcf $O/txpmcw 4194304 $O/pmc_c4tx.json tx_kernel=1+33 > $O/pmct_c4tx.log 2>&1
    for rep in 1 2; do
      timeout -k 10 200 python tools/txbench.py 1048576 24 1 --rotate 8 --rings 4 > $O/txb_4x1M_$rep.log 2>&1 || exit 1
      timeout -k 10 200 python tools/txbench.py 1048576 24 1 --rotate 4 --concat 2 --rings 4 > $O/txb_4x2M_$rep.log 2>&1 || exit 1
      for v in 4x1M 4x2M; do echo "$v $(tail -1 $O/txb_${v}_$rep.log)"; done
    done
    ;;
  r05aj)
    # up to eight consecutive rings per tx launch: the tx / parity / window /
    # group GPU tests, a multi-ring fuzz (2-8 rings), txbench at 4 and 8 rings,
    # the bench's c4tx line at 4 and 8, rocprof + PMC of the 8-ring launch
    TESTS="tests/test_gpu_tx.py tests/test_gpu_parity.py tests/test_gpu_window.py tests/test_gpu_group.py" \
      bash tools/gpu.sh $S testsall || exit 1
    timeout -k 10 240 python -u tools/fuzz_multi_ring.py 3000 100 3000 > $O/fuzz.log 2>&1 || { tail -3 $O/fuzz.log; exit 1; }
    tail -1 $O/fuzz.log
    for r in 4 8; do
      timeout -k 10 200 python tools/txbench.py 1048576 24 1 --rotate 8 --rings $r > $O/txb_r$r.log 2>&1 || exit 1
      echo "rings=$r $(tail -1 $O/txb_r$r.log)"
      BENCH_ARGS="--steps 10 --warmup 3 --extras c4tx --no-cpu-baseline --tx-rings $r" bash tools/gpu.sh $S bench || exit 1
      mv $O/bench.log $O/bench_tx$r.log
    done
    TXB_ARGS="1048576 24 1 --rotate 8 --rings 8" bash tools/gpu.sh $S txprof txpmc || exit 1
    python3 tools/pmc_traffic.py $O/txpmcf $O/txpmcw 8388608 $O/pmc_c4tx.json tx_kernel=1+33 > $O/pmct_c4tx.log 2>&1
    ;;
  r05ak)
    # what bounds the tx kernel at eight rings per launch (8192 tiles, eight
    # generations at four workgroups per CU): SQ instruction mix, busy and
    # wait cycles, LDS bank conflicts (two passes of txbench --rings 8)
    TX="tools/txbench.py 1048576 12 1 --rotate 8 --rings 8"
    sq_pass sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
      python3 $TX
    sq_pass sq2 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
      python3 $TX
    python3 tools/pmc_summary.py $O/sq1 $O/sq2 > $O/sq_summary.txt 2>&1 || true
    cat $O/sq_summary.txt
    ;;
  r05al)
    # final tree (eight tx rings per launch): the suite, smoke, the bench as
    # the driver runs it, rocprof of the bench, PMC of c5 / c2 / c3 / c4 and
    # of the 8-ring tx launch
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    bash tools/gpu.sh $S rocprof || exit 1
    PMC_CFGS="c5 c2 c3 c4" bash tools/gpu.sh $S pmc || exit 1
    TXB_ARGS="1048576 24 1 --rotate 8 --rings 8" bash tools/gpu.sh $S txprof txpmc || exit 1
    python3 tools/pmc_traffic.py $O/txpmcf $O/txpmcw 8388608 $O/pmc_c4tx.json tx_kernel=1+33 > $O/pmct_c4tx.log 2>&1
    ;;
  r05am)
    # c3's launch shape (the poll round's 8 rings of 256K IMIX frames): calls
    # of 4 on 2 streams (the bench's) against one call of 8 on 1 stream and
    # calls of 8 on 2 streams, alternated
    for rep in 1 2; do
      for v in "4 2" "8 1" "8 2"; do
        set -- $v
        timeout -k 10 300 python bench.py --config c3 --no-extra --no-cpu-baseline --steps 40 --warmup 5 \
          --rings-per-launch $1 --streams $2 > $O/c3_p$1_s$2_$rep.log 2>&1 || exit 1
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d.get('end_to_end_mpps'), r['frac'], r.get('kernel_us_median'), d['config'])" \
          $O/c3_p$1_s$2_$rep.log "p=$1 s=$2" || exit 1
      done
    done
    ;;
  r05an)
    # more multi-ring tx fuzzing on the final tree: 200 seeds of 5000 events,
    # and 100 over a table past LDS (3000 filler rules: U and X probes)
    timeout -k 10 400 python -u tools/fuzz_multi_ring.py 5000 200 5000 > $O/fuzz.log 2>&1 || { tail -3 $O/fuzz.log; exit 1; }
    tail -1 $O/fuzz.log
    timeout -k 10 400 python -u tools/fuzz_multi_ring.py 6000 100 3000 3000 > $O/fuzz_filler.log 2>&1 || { tail -3 $O/fuzz_filler.log; exit 1; }
    tail -1 $O/fuzz_filler.log
    ;;
  r05ao)
    # c5's scatter (2 x 8M per call: 2048 chunks of 8 tiles = 2.67 generations
    # of 768 resident) at 4-tile chunks (4096 chunks, 5.3 generations: a
    # finer tail), the test build's USN_SCATTER_TC, alternated
    for rep in 1 2; do
      for tc in 8 4; do
        USN_SCATTER_TC=$tc timeout -k 10 300 python tools/scatter_bench.py --config c5 --frames 8388608 --multi 2 \
          base testlib > $O/scb_c5_tc${tc}_$rep.log 2>&1 || exit 1
        echo "tc=$tc"; grep scatter $O/scb_c5_tc${tc}_$rep.log
      done
    done
    ;;
  r05ap)
    # the share of the key1 / key2 probes (hashes + slot reads) in the 8-ring
    # tx launch: build/abl/txnoprobe (no K1/K2 probes, wrong decisions)
    # against build/abl/base, alternated
    for rep in 1 2; do
      for v in base txnoprobe; do
        timeout -k 10 200 python tools/txbench.py 1048576 24 1 build/abl/$v/libusn.so --rotate 8 --rings 8 \
          > $O/txb_${v}_$rep.log 2>&1 || exit 1
        echo "$v $(tail -1 $O/txb_${v}_$rep.log)"
      done
    done
    ;;
  r05aq)
    # final tree again (product library rebuilt after the hash A/B was
    # reverted; same sources as r05al): the suite, smoke, the driver's bench
    bash tools/gpu.sh $S testsall || exit 1
    bash tools/gpu.sh $S smoke || exit 1
    BENCH_ARGS="--steps 40 --warmup 5" bash tools/gpu.sh $S bench || exit 1
    ;;
  r05ar)
    # eight 1M rings of distinct flows in one tx grid, every ring learning
    TESTS=tests/test_gpu_tx.py TEST_K="eight_rings_all_learn" bash tools/gpu.sh $S testsall || exit 1
    ;;
  r05at)
    # HEAD (r05as's tree): more multi-ring tx fuzz on new seeds (plain, and
    # with an image past LDS so the rx kernel probes U and X), then c5's
    # FETCH/WRITE passes on this tree
    timeout -k 10 500 python -u tools/fuzz_multi_ring.py 7000 300 5000 > $O/fuzz.log 2>&1 || { tail -3 $O/fuzz.log; exit 1; }
    tail -1 $O/fuzz.log
    timeout -k 10 400 python -u tools/fuzz_multi_ring.py 8000 150 3000 3000 > $O/fuzz_filler.log 2>&1 || { tail -3 $O/fuzz_filler.log; exit 1; }
    tail -1 $O/fuzz_filler.log
    PMC_CFGS="c5" bash tools/gpu.sh $S pmc || exit 1
    ;;
  r05au)
    # 16-tile scatter chunks (two consecutive tiles per wave, 2 workgroups per
    # CU; the test build's USN_SCATTER_TC=16) against the product's 8: scan +
    # scatter device time and lists equal to the product's, c5 2 x 8M, c4 and
    # c2 8 x 1M; then the ballot fallback forced (USN_SCATTER_SLOW_RANK)
    mkdir -p build/abl/testlib && cp build/test/libusn.so build/abl/testlib/libusn.so
    for rep in 1 2; do
      for c in c5 c4 c2; do
        if [ $c = c5 ]; then A="--frames 8388608 --multi 2"; else A="--frames 1048576 --multi 8"; fi
        USN_SCATTER_TC=16 timeout -k 10 300 python tools/scatter_bench.py --config $c $A \
          --json $O/scb_${c}_$rep.json base testlib > $O/scb_${c}_$rep.log 2>&1 || { tail -3 $O/scb_${c}_$rep.log; exit 1; }
        echo "$c rep $rep"; grep scatter $O/scb_${c}_$rep.log
      done
    done
    USN_SCATTER_TC=16 USN_SCATTER_SLOW_RANK=1 timeout -k 10 300 python tools/scatter_bench.py --config c5 \
      --frames 8388608 --multi 2 --launches 5 base testlib > $O/scb_c5_slow.log 2>&1 || { tail -3 $O/scb_c5_slow.log; exit 1; }
    echo "c5 forced fallback"; grep scatter $O/scb_c5_slow.log
    ;;
  r05av)
    # the scatter compiled for 8 waves per SIMD (64 VGPRs, 96 B of spills per
    # lane; build/abl/scwpe8) against the product's 6 (80 VGPRs): launches of
    # few bins (c2: 32.5 KiB of LDS) fit 4 workgroups per CU by LDS; c5 stays
    # at 3 (52.9 KiB)
    for rep in 1 2; do
      for c in c2 c4 c5; do
        if [ $c = c5 ]; then A="--frames 8388608 --multi 2"; else A="--frames 1048576 --multi 8"; fi
        timeout -k 10 300 python tools/scatter_bench.py --config $c $A \
          --json $O/scb_${c}_$rep.json base scwpe8 > $O/scb_${c}_$rep.log 2>&1 || { tail -3 $O/scb_${c}_$rep.log; exit 1; }
        echo "$c rep $rep"; grep scatter $O/scb_${c}_$rep.log
      done
    done
    ;;
  r05ax)
    # the scatter without spills (the fallback's lane opaque to the compiler:
    # 71 VGPRs, no scratch, against 80 and 32 B of spill stores per lane):
    # the scatter and volume GPU tests; scan + scatter time against HEAD~
    # (build/abl/spill) and the spill-free build at 8 waves per SIMD
    # (build/abl/scwpe8: 64 VGPRs, no scratch now); the ballot fallback forced
    TESTS="tests/test_gpu_scatter.py tests/test_gpu_volume.py" bash tools/gpu.sh $S testsall || exit 1
    for rep in 1 2; do
      for c in c5 c4 c2; do
        if [ $c = c5 ]; then A="--frames 8388608 --multi 2"; else A="--frames 1048576 --multi 8"; fi
        timeout -k 10 300 python tools/scatter_bench.py --config $c $A \
          --json $O/scb_${c}_$rep.json base spill scwpe8 > $O/scb_${c}_$rep.log 2>&1 || { tail -3 $O/scb_${c}_$rep.log; exit 1; }
        echo "$c rep $rep"; grep scatter $O/scb_${c}_$rep.log
      done
    done
    USN_SCATTER_SLOW_RANK=1 timeout -k 10 300 python tools/scatter_bench.py --config c5 \
      --frames 8388608 --multi 2 --launches 5 base testlib > $O/scb_c5_slow.log 2>&1 || { tail -3 $O/scb_c5_slow.log; exit 1; }
    echo "c5 forced fallback"; grep scatter $O/scb_c5_slow.log
    ;;
  *) echo "unknown session $S"; exit 2 ;;
esac
echo "== session $S done"
