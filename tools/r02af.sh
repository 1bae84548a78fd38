# r02af: tx head decisions published per tile; bench ramp order check
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02af
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-3} | cut -c1-220; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest_tx 600 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_group.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
step txbench 300 python tools/txbench.py 1048576 12 1
TAILN=22 step txstamps 200 python tools/stamps.py c4tx 1048576
step b20 300 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline
step b400 300 python bench.py --steps 400 --warmup 5 --no-extra --no-cpu-baseline
exit 0
