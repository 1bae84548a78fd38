# r02ah: persistent classify grid (USN_PERSIST) A/B; parity
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ah
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20" $O/$name.log | tail -${TAILN:-8}; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_volume.py tests/test_gpu_window.py -x -q --timeout 300 --timeout-method thread
step abl_c5_8m 400 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 3 --launches 30 base persistoff
step abl_c4_8m 400 python tools/abl.py --config c4 --frames 8388608 --batches 2 --rounds 3 --launches 30 base persistoff
step abl_c2_8x1m 400 python tools/abl.py --config c2 --frames 1048576 --multi 8 --batches 2 --rounds 3 --launches 30 base persistoff
step abl_c3 400 python tools/abl.py --config c3 --frames 1048576 --batches 2 --rounds 3 --launches 30 base persistoff
step bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
exit 0
