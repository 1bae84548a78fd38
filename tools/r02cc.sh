# r02cc: bench variance at 2 vs 8 rx queues per step (20 timed steps each, three runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02cc
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -1 $O/$name.log | cut -c1-160; fatal $rc && exit $rc; return 0; }
for i in 1 2 3; do
  step q2_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra
  step q8_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --queues 8
done
exit 0
