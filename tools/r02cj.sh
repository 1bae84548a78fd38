# r02cj: spread of the default bench shape on one box (5 x 20 steps, 2 x 100 steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02cj
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; fatal $rc && exit $rc; return 0; }
for i in 1 2 3 4 5; do
  step b20_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
done
for i in 1 2; do
  step b100_$i 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-extra
done
exit 0
