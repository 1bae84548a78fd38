# r02ae: bench ramp order check; tx back to LAST after the prefix pass
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ae
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -h "^{" $O/$name.log | cut -c1-200; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc; return 0; }
step txbench 300 python tools/txbench.py 1048576 12 1
step b20 300 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline
step b400 300 python bench.py --steps 400 --warmup 5 --no-extra --no-cpu-baseline
step b20b 300 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline
exit 0
