# r02cn: A/B non-temporal length loads against base, c5 / c4 / c2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02cn
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-6} $O/$name.log | cut -c1-300; fatal $rc && exit $rc; return 0; }
step abl_c5 300 python tools/abl.py --config c5 --frames 8388608 --batches 2 --multi 2 --rounds 5 --launches 40 base lennt base lennt
step abl_c4 300 python tools/abl.py --config c4 --frames 8388608 --batches 2 --rounds 5 --launches 40 base lennt base lennt
step abl_c2 300 python tools/abl.py --config c2 --frames 1048576 --batches 8 --multi 8 --rounds 5 --launches 40 base lennt base lennt
exit 0
