# r02ak: tx phase 1 pipelined (rounds' header loads together, lengths first,
# LDS bridge/listen lookups, displacement reads per round); parity + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ak
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20" $O/$name.log | tail -${TAILN:-8}; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest_tx 600 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 300 --timeout-method thread
TAILN=3 step tx_base 200 python tools/txbench.py 1048576 8 1
TAILN=3 step tx_pipeoff 200 python tools/txbench.py 1048576 8 1 build/abl/txpipeoff/libusn.so
TAILN=3 step tx_noprobe 200 python tools/txbench.py 1048576 8 1 build/abl/txnoprobe/libusn.so
TAILN=30 step stamps_c4tx 200 python tools/stamps.py c4tx 1048576
TAILN=30 STAMPS512=1 step stamps_c5 200 python tools/stamps.py c5 8388608
exit 0
