# r02am: after the one-pass fix (46 VGPRs again): base vs tiles-per-workgroup (capped at 64 VGPRs); minimal stamps; bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02am
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20" $O/$name.log | tail -${TAILN:-8}; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc; return 0; }
step abl_c5_8m 400 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 3 --launches 30 base persist2 persist4 persist
TAILN=3 STAMPS512=1 STAMPS_BUILD=stampmin step stampmin_c5 200 python tools/stamps.py c5 8388608
step bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
exit 0
