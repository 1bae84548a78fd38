# r02t: c3 line-granular floor, c3 A/B, PMC traffic of the bench configs (c5, c2)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02t
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20" $O/$name.log | tail -${TAILN:-8}; fatal $rc && exit $rc; return 0; }
step floor2048 200 build/stride_floor 4194304 2048 30
step floor64 200 build/stride_floor 4194304 64 30
step abl_c3 400 python tools/abl.py --config c3 --frames 1048576 --batches 4 --rounds 3 base loadonly noprobe nosort
for c in c5 c2; do
  rm -rf $O/pmcf_$c $O/pmcw_$c
  step pmcf_$c 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcf_$c -o run -- python3 bench.py --config $c --no-extra --steps 16 --warmup 4 --no-cpu-baseline --launch-probe 0
  step pmcw_$c 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmcw_$c -o run -- python3 bench.py --config $c --no-extra --steps 16 --warmup 4 --no-cpu-baseline --launch-probe 0
  step pmct_$c 60 python3 tools/pmc_traffic.py $O/pmcf_$c $O/pmcw_$c 8388608 $O/pmc_$c.json
done
STEPS=pmccfg PMC_CFGS=c3 bash tools/gpu_check.sh > $O/pmccfg_c3.log 2>&1; echo "== pmccfg rc=$?"; tail -20 $O/pmccfg_c3.log
exit 0
