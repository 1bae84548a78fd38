# r02u: 48-byte lane-path reads (c3) and tx header reads; parity
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02u
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-8}; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc; return 0; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tx.py tests/test_gpu_window.py -x -q --timeout 120 --timeout-method thread
step abl_c3 400 python tools/abl.py --config c3 --frames 1048576 --batches 4 --rounds 3 base loadonly
step txbench 200 python tools/txbench.py 1048576 12 1
step floor64 200 build/stride_floor 4194304 64 30
exit 0
