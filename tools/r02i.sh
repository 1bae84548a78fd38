# r02i: LDS displacements at 3 workgroups per CU (radix keys in the stage), A/B at 1M and 8M
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02i
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/r02i/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU" gpurun_out/r02i/$name.log | tail -${TAILN:-9}; fatal $rc && exit $rc; return 0; }
step abl_c5 400 python tools/abl.py --config c5 --rounds 3 base disp16 disp16nb disp16@USN_T512=0 noprobe
step abl_c5_8m 400 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 3 --launches 30 base disp16 disp16nb noprobe
step abl_c4 400 python tools/abl.py --config c4 --rounds 3 base disp16 noprobe
step abl_c4_8m 400 python tools/abl.py --config c4 --frames 8388608 --batches 2 --rounds 3 --launches 30 base disp16 noprobe
exit 0
