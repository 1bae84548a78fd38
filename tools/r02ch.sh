# r02ch: measurement set with both c5 rings in one launch (the bench default now): bench, rocprof, PMC per 16M-frame launch, every config, 2-rank run
# PMC traffic (c5, c2), tx, host loop, every config
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ch
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-4} | cut -c1-400; fatal $rc && exit $rc; return 0; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 5
TAILN=2 step bench_n2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline
rm -rf $O/prof
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --ramp 40
step trace_summary 60 python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv
for c in c5 c2; do
  if [ $c = c5 ]; then F=16777216; else F=8388608; fi
  rm -rf $O/pmcf_$c $O/pmcw_$c
  step pmcf_$c 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcf_$c -o run -- python3 bench.py --config $c --no-extra --steps 16 --warmup 4 --no-cpu-baseline --launch-probe 0 --ramp 0
  step pmcw_$c 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmcw_$c -o run -- python3 bench.py --config $c --no-extra --steps 16 --warmup 4 --no-cpu-baseline --launch-probe 0 --ramp 0
  step pmct_$c 60 python3 tools/pmc_traffic.py $O/pmcf_$c $O/pmcw_$c $F $O/pmc_$c.json
done
step txbench 300 python tools/txbench.py 1048576 12 1
rm -rf $O/txprof
step txprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/txprof -o run -- python3 tools/txbench.py 1048576 24 1
step tx_summary 60 python3 tools/trace_summary.py $O/txprof/run_kernel_trace.csv
step hostio 300 python tools/hostio.py c2 1048576 8 4 6
step allcfg 1100 python tools/all_configs.py --out $O/all_configs.json
exit 0
