# r02bc: projection streams (fixed filler owner); c5 / c4tx phase stamps (512-thread build)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bc
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-4} | cut -c1-400; fatal $rc && exit $rc; return 0; }
step pytest_proj 300 python -u -m pytest tests/test_gpu_parity.py -k projection -m gpu -q --timeout 300 --timeout-method thread
export STAMPS512=1
TAILN=30 step stamps_c5 300 python tools/stamps.py c5 8388608
TAILN=30 step stamps_c4tx 300 python tools/stamps.py c4tx 1048576
exit 0
