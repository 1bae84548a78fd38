# r02bb: full GPU suite on the projection-table tree; c5 / c4tx phase stamps; tx bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bb
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-4} | cut -c1-400; fatal $rc && exit $rc; return 0; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
TAILN=16 step stamps_c5 300 python tools/stamps.py c5 8388608
TAILN=16 step stamps_c4tx 300 python tools/stamps.py c4tx 1048576
step txbench 300 python tools/txbench.py 1048576 12 1
exit 0
