# r02j: 48-byte header stage; LDS displacements at 3 (group 8) and 4 (group 10) workgroups per CU
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02j
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/r02j/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU" gpurun_out/r02j/$name.log | tail -${TAILN:-9}; fatal $rc && exit $rc; return 0; }
step abl_c5_8m 400 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 3 --launches 30 base disp16 disp16@USN_PH_GROUP=10,USN_PH_LOAD=0.75 noprobe
step abl_c5 400 python tools/abl.py --config c5 --rounds 3 base disp16 disp16@USN_PH_GROUP=10,USN_PH_LOAD=0.75
step abl_c4_8m 400 python tools/abl.py --config c4 --frames 8388608 --batches 2 --rounds 3 --launches 30 base noprobe
step abl_c2_8m 400 python tools/abl.py --config c2 --frames 8388608 --batches 2 --rounds 3 --launches 30 base noprobe
step pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_window.py -x -q --timeout 120 --timeout-method thread
exit 0
