# r02bt: tx end to end (classify call + usn_finalize wall time): steady 1M / 8M rings, learning rings (4 distinct)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bt
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-1} $O/$name.log | cut -c1-400; fatal $rc && exit $rc; return 0; }
step tx_1m 300 python tools/txbench.py 1048576 12 1
step tx_8m 300 python tools/txbench.py 8388608 8 1
TAILN=14 step tx_learn_1m 300 python tools/txbench.py 1048576 12 4
exit 0
