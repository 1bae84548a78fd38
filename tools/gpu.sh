#!/bin/bash
# The one GPU-session runner (replaces round 2's per-experiment tools/r02*.sh).
#   tools/gpu.sh TAG STEP [STEP ...]      output: gpurun_out/TAG/<step>.log
# Each step runs under its own time limit; the session stops at the first
# fault / abort / time limit (exit >= 124, 134, 139).  Plain test failures
# (exit 1) do not stop later steps.  Knobs per step come from the environment
# (TESTS, TEST_K, BENCH_ARGS, PMC_CFGS, ABL_ARGS, ABL_VARIANTS, TXB_ARGS, ...).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "-- $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" "$O/$name.log" | tail -n ${TAILN:-4} | cut -c1-400
  if fatal $rc; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
pmc_pass() {  # pmc_pass NAME COUNTERS CMD...
  local name=$1 ctr=$2; shift 2
  rm -rf $O/$name
  step $name 300 timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$name -o run -- "$@"
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 1100 python -u -m pytest ${TESTS:-tests} -m gpu -q -x -rf --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"} ;;
    testsall) step pytest_gpu 1100 python -u -m pytest ${TESTS:-tests} -m gpu -q -rf --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"} ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} ;;
    bench_n2) TAILN=2 step bench_n2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-extra ;;
    rocprof) rm -rf $O/prof
      step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --ramp 40 ${ROCPROF_ARGS:-}
      step trace_summary 60 python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv ;;
    pmc)  # FETCH_SIZE / WRITE_SIZE passes per config of PMC_CFGS through bench.py's launch shape
      for c in ${PMC_CFGS:-c5 c2}; do
        # the launch shape the bench line uses for the config (c3: its 8 queues)
        QA=$(python3 -c "import bench; q = bench.extra_queues('$c'); print('--queues %d' % q if q else '')")
        F=$(python3 -c "import bench; print(bench.launch_frames('$c', bench.extra_queues('$c')))")
        pmc_pass pmcf_$c FETCH_SIZE python3 bench.py --config $c $QA --no-extra --steps 16 --warmup 4 --no-cpu-baseline --launch-probe 0 --ramp 0
        pmc_pass pmcw_$c WRITE_SIZE python3 bench.py --config $c $QA --no-extra --steps 16 --warmup 4 --no-cpu-baseline --launch-probe 0 --ramp 0
        FF=""; [ $c = c3 ] && FF="classify_rx_kernel=1"   # one 64-B request per 2048-B slot
        step pmct_$c 60 python3 tools/pmc_traffic.py $O/pmcf_$c $O/pmcw_$c $F $O/pmc_$c.json $FF
      done ;;
    txbench) step txbench 300 python tools/txbench.py ${TXB_ARGS:-1048576 12 1} ;;
    txprof) rm -rf $O/txprof
      step txprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/txprof -o run -- python3 tools/txbench.py ${TXB_ARGS:-1048576 24 1}
      step tx_summary 60 python3 tools/trace_summary.py $O/txprof/run_kernel_trace.csv ;;
    txpmc)
      pmc_pass txpmcf FETCH_SIZE python3 tools/txbench.py ${TXB_ARGS:-1048576 24 1}
      pmc_pass txpmcw WRITE_SIZE python3 tools/txbench.py ${TXB_ARGS:-1048576 24 1} ;;
    hostio) step hostio 300 python tools/hostio.py ${HOSTIO_ARGS:-c2 1048576 8 4 6} ;;
    allcfg) step allcfg 1100 python tools/all_configs.py --out $O/all_configs.json ${ALLCFG_ARGS:-} ;;
    abl) for c in ${ABL_CFGS:-c5}; do
        step abl_$c 600 python tools/abl.py --config $c --json $O/abl_$c.json ${ABL_ARGS:-} ${ABL_VARIANTS:-base}
      done ;;
    scb) for c in ${SCB_CFGS:-c5 c2}; do
        if [ $c = c5 ]; then A="--frames 8388608 --multi 2"; else A="--frames 1048576 --multi 8"; fi
        step scb_$c 300 python tools/scatter_bench.py --config $c $A --json $O/scb_$c.json ${SCB_VARIANTS:-base}
      done ;;
    stamps) step stamps 300 python tools/stamps.py ${STAMP_ARGS:-c5} ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done"
