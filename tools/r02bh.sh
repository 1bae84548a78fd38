# r02bh: lane path reads bytes 12..43 in two dword-aligned 16-byte loads: parity, A/B c3 (2048-byte slots)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bh
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-4} | cut -c1-400; fatal $rc && exit $rc; return 0; }
step pytest_par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_volume.py tests/test_gpu_window.py -m gpu -x -q --timeout 300 --timeout-method thread
step abl_c3 300 python tools/abl.py --config c3 --frames 1048576 --batches 2 --rounds 5 --launches 40 base lane48
step abl_c3b 300 python tools/abl.py --config c3 --frames 1048576 --batches 2 --rounds 5 --launches 40 lane48 base
exit 0
