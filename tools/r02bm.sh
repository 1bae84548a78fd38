# r02bm: c5 ablation ladder and phase stamps on the final kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bm
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-4} | cut -c1-400; fatal $rc && exit $rc; return 0; }
TAILN=6 step abl_c5 300 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 5 --launches 40 base noprobe nosort loadonly nodispcopy
export STAMPS512=1
TAILN=30 step stamps_c5 300 python tools/stamps.py c5 8388608
exit 0
