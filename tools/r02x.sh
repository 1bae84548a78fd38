# r02x: bench launch shapes for c5 (2 queues of 8M per step)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02x
mkdir -p $O
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep '^{' $O/$name.log | python3 -c "import json,sys; b=json.loads(sys.stdin.read()); print(b['value'], b['ms_per_step'], b['config'].get('streams'), b['config'].get('batches_per_launch'), b['roofline'].get('kernel_us_median'))"; fatal $rc && exit $rc; return 0; }
A="--no-extra --no-cpu-baseline --steps 20 --warmup 5"
step s2p1 300 python bench.py $A
step s1p1 300 python bench.py $A --streams 1 --queues 2
step s1p2 300 python bench.py $A --streams 1 --queues 2 --rings-per-launch 2
step s2p1_q4 300 python bench.py $A --queues 4
step s2p2_q4 300 python bench.py $A --queues 4 --rings-per-launch 2
exit 0
