# r02y: c5 8M budget on the current kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02y
mkdir -p $O
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20" $O/$name.log | tail -${TAILN:-8}; fatal $rc && exit $rc; return 0; }
step abl_c5_8m 400 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 3 --launches 30 base noprobe nosort loadonly
step abl_c2_8m 400 python tools/abl.py --config c2 --frames 8388608 --batches 2 --rounds 3 --launches 30 base nosort loadonly
STAMPS512=1 step stamps_c5 300 python tools/stamps.py c5 8388608
exit 0
