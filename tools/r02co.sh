# r02co: final check of the round's tree: GPU parity suite, smoke, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02co
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-3} $O/$name.log | cut -c1-400; fatal $rc && exit $rc; return 0; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 600 python bench.py
exit 0
