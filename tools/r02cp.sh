# r02cp: A/B non-temporal per-lane header loads (USN_LOAD_NT: the lane path, c3; the tx header loads) against base
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02cp
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-4} $O/$name.log | cut -c1-300; fatal $rc && exit $rc; return 0; }
step abl_c3 300 python tools/abl.py --config c3 --frames 262144 --batches 8 --multi 8 --rounds 5 --launches 40 base loadnt
step abl_c5 300 python tools/abl.py --config c5 --frames 8388608 --batches 2 --multi 2 --rounds 5 --launches 40 base loadnt
for i in 1 2 3; do
  TAILN=1 step tx_base_$i 300 python tools/txbench.py 1048576 24 1 build/abl/base/libusn.so
  TAILN=1 step tx_nt_$i 300 python tools/txbench.py 1048576 24 1 build/abl/loadnt/libusn.so
done
exit 0
