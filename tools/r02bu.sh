# r02bu: c5x (connected rules on listening ports: the overflow table's worst case): parity, A/B vs no U
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bu
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-4} | cut -c1-400; fatal $rc && exit $rc; return 0; }
step pytest_c5x 300 python -u -m pytest tests/test_gpu_parity.py -k "c5x" -m gpu -x -q --timeout 300 --timeout-method thread
step abl_c5x 300 python tools/abl.py --config c5x --frames 8388608 --batches 2 --rounds 5 --launches 40 base base@USN_NO_PROJ=1
exit 0
