# r02cr: A/B slot load of the image (USN_PH_LOAD 0.65 default, 0.8, 0.9): a smaller projection table, c5 / c4
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02cr
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-6} $O/$name.log | cut -c1-300; fatal $rc && exit $rc; return 0; }
V="base@USN_PH_LOAD=0.65 base@USN_PH_LOAD=0.8 base@USN_PH_LOAD=0.9"
step abl_c5 300 python tools/abl.py --config c5 --frames 8388608 --batches 2 --multi 2 --rounds 5 --launches 40 $V
step abl_c4 300 python tools/abl.py --config c4 --frames 8388608 --batches 2 --rounds 5 --launches 40 $V
exit 0
