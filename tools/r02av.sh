# r02av: cross-tile L2 prefetch (tile w + d touched by tile w's workgroup) A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02av
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20" $O/$name.log | tail -${TAILN:-8}; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc; return 0; }
step abl_c5_8m 600 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 4 --launches 30 base pf512 pf1024 pf2048
step abl_c2_8m 600 python tools/abl.py --config c2 --frames 8388608 --batches 2 --rounds 4 --launches 30 base pf1024
exit 0
