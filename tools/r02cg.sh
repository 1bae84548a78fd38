# r02cg: bench step shapes: 2 rings on 2 streams (default) vs both rings in one launch on one stream
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02cg
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; fatal $rc && exit $rc; return 0; }
for i in 1 2 3; do
  step s2_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
  step s1m2_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --streams 1 --rings-per-launch 2
  step s2m2_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --queues 4 --rings-per-launch 2
done
exit 0
