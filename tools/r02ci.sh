# r02ci: every config with the bench's launch shapes (c5: both rings in one launch), two default bench repeats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ci
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; fatal $rc && exit $rc; return 0; }
step allcfg 900 python -u tools/all_configs.py --out $O/all_configs.json
step bench1 300 python bench.py
step bench2 300 python bench.py
exit 0
