# r02br: nt output stores only for L2-resident images (c4, c5), plain for LDS images (c2): parity, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02br
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-4} | cut -c1-400; fatal $rc && exit $rc; return 0; }
step pytest_par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_volume.py -m gpu -x -q --timeout 300 --timeout-method thread
step abl_c5 300 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 5 --launches 40 base storetemp
step abl_c5b 300 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 5 --launches 40 storetemp base
step abl_c4 300 python tools/abl.py --config c4 --frames 8388608 --batches 2 --rounds 5 --launches 40 base storetemp
step abl_c2 300 python tools/abl.py --config c2 --frames 1048576 --batches 8 --multi 8 --rounds 5 --launches 40 base storetemp
exit 0
