# r02bv: parallel image build (registry scan, shard partition, in-place placement; groups of 5
# beyond 128 K keys): full GPU suite, tx learning rings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bv
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state" $O/$name.log | tail -${TAILN:-4} | cut -c1-300; fatal $rc && exit $rc; return 0; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
TAILN=14 step tx_learn_1m 300 python tools/txbench.py 1048576 12 4
step tx_1m 300 python tools/txbench.py 1048576 12 1
exit 0
