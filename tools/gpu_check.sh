#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Stops at the first fault / abort / timeout (exit >= 124); plain test
# failures (exit 1) do not stop the later measurement steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal rc=$rc in $name: stopping"; exit $rc
  fi
  return 0
}
for s in ${STEPS:-tests smoke bench prof}; do
  case $s in
    tests) step pytest_gpu 900 python -m pytest tests -m gpu -q -x -rf ;;
    testsall) step pytest_gpu 900 python -m pytest tests -m gpu -q -rf ;;
    txtests) step pytest_tx 900 python -m pytest tests/test_gpu_tx.py tests/test_gpu_parity.py -m gpu -q -rf -k "${TX_K:-tx or kat or random}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof) rm -rf gpurun_out/prof; step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 400 --warmup 40 --no-cpu-baseline ;;
    abl) step abl 600 python tools/abl.py --json gpurun_out/abl.json ${ABL_ARGS:-} ;;
    stamps) step stamps 300 python tools/stamps.py ${STAMP_ARGS:-c2} ;;
    ablms) step ablms 600 python tools/abl.py --streams ${NSTREAMS:-2} --batches 6 --json gpurun_out/ablms.json ${ABL_VARIANTS:-base loadonly} ;;
    ablmulti) step ablmulti_${NMULTI:-4}_${NSTREAMS:-1} 600 python tools/abl.py --multi ${NMULTI:-4} --streams ${NSTREAMS:-1} --batches ${NBATCH:-8} --json gpurun_out/ablmulti.json ${ABL_VARIANTS:-base loadonly} ;;
    hostio) step hostio 300 python tools/hostio.py ${HOSTIO_ARGS:-} ;;
    txbench) step txbench 600 python tools/txbench.py ${TXB_ARGS:-} ;;
    ablcfg)  # rx A/B of ABL_VARIANTS per config of ABL_CFGS (one process per config)
      for c in ${ABL_CFGS:-c4 c5}; do
        step abl_$c 600 python tools/abl.py --config $c --rounds 3 --json gpurun_out/abl_$c.json ${ABL_VARIANTS:-old new}
      done ;;
    txab)   # tx A/B: the same txbench per A/B build (make abl)
      for v in ${TXAB_VARIANTS:-base t512}; do
        step txab_$v 300 python tools/txbench.py 1048576 12 1 build/abl/$v/libusn.so
      done ;;
    allcfg) step allcfg 1100 python tools/all_configs.py ${ALLCFG_ARGS:-} ;;
    txprof) rm -rf gpurun_out/txprof; step txprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/txprof -o run -- python3 tools/txbench.py ${TXB_ARGS:-} ;;
    ablsmall) step ablsmall 600 python tools/abl.py --frames 131072 --batches 1 --json gpurun_out/ablsmall.json ;;
    counters)
      step listctr 120 rocprofv3 -L
      i=0
      for set in ${PMC_SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"} \
                 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
                 "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
                 "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"; do
        i=$((i+1))
        step pmc$i 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/kbench.py ${KB_ARGS:-c2 1048576 30}
      done
      step pmcsum 60 python3 tools/pmc_summary.py gpurun_out/pmc ;;
    pmccfg)  # per config: kernel trace + FETCH_SIZE / WRITE_SIZE / L2 hit-miss passes (kbench launches)
      for c in ${PMC_CFGS:-c3 c4 c5}; do
        rm -rf gpurun_out/pmccfg/$c
        step kt_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmccfg/$c/kt -o run -- python3 tools/kbench.py $c ${KB_FRAMES:-1048576} 40
        j=0
        for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
          j=$((j+1))
          step pmc_${c}_$j 300 timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmccfg/$c/p$j -o run -- python3 tools/kbench.py $c ${KB_FRAMES:-1048576} 30
        done
        step pmcsum_$c 60 python3 tools/pmc_summary.py gpurun_out/pmccfg/$c/p1 gpurun_out/pmccfg/$c/p2 gpurun_out/pmccfg/$c/p3 gpurun_out/pmccfg/$c/p4
      done ;;
    traffic)
      rm -rf gpurun_out/pmcf gpurun_out/pmcw
      step pmcf 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf -o run -- python3 bench.py --steps 64 --warmup 8 --no-cpu-baseline --launch-probe 0
      step pmcw 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw -o run -- python3 bench.py --steps 64 --warmup 8 --no-cpu-baseline --launch-probe 0
      step pmctraffic 60 python3 tools/pmc_traffic.py gpurun_out/pmcf gpurun_out/pmcw ${PMC_FRAMES:-8388608} gpurun_out/pmc_c2.json ;;
  esac
done
echo "=== done"
