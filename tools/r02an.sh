# r02an: the tx kernel at 512 threads per tile (USN_TX_T512=1): parity + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02an
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20" $O/$name.log | tail -${TAILN:-8}; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc; return 0; }
TAILN=2 step tx256 200 python tools/txbench.py 1048576 8 1
TAILN=2 USN_TX_T512=1 step tx512 200 python tools/txbench.py 1048576 8 1
USN_TX_T512=1 step pytest_tx512 600 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 300 --timeout-method thread
TAILN=30 USN_TX_T512=1 STAMPS512=1 step stamps_c4tx512 200 python tools/stamps.py c4tx 1048576
exit 0
