# r02ca: byte-row sort stores each order entry directly (no LDS order row, one barrier and readback fewer)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ca
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state" $O/$name.log | tail -${TAILN:-4} | cut -c1-300; fatal $rc && exit $rc; return 0; }
step pytest_par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_volume.py -m gpu -x -q --timeout 300 --timeout-method thread
step abl_c5 300 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 5 --launches 40 base orderlds
step abl_c5b 300 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 5 --launches 40 orderlds base
step abl_c4 300 python tools/abl.py --config c4 --frames 8388608 --batches 2 --rounds 5 --launches 40 base orderlds
exit 0
