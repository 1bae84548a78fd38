# r02cb: bench repeat on the final tree (box-to-box variance of the headline), smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02cb
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-1} $O/$name.log | cut -c1-200; fatal $rc && exit $rc; return 0; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do step bench_$i 600 python bench.py --steps 20 --warmup 5; done
exit 0
