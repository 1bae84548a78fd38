# r02bi: tx EARLY look-back overlapped with the LAST walk back: tx parity, A/B (alternating txbench)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bi
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-4} | cut -c1-400; fatal $rc && exit $rc; return 0; }
step pytest_tx 600 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_group.py -m gpu -x -q --timeout 300 --timeout-method thread
for i in 1 2 3; do
  TAILN=1 step tx_base_$i 300 python tools/txbench.py 1048576 48 1 build/abl/base/libusn.so
  TAILN=1 step tx_off_$i 300 python tools/txbench.py 1048576 48 1 build/abl/txearlyoff/libusn.so
done
exit 0
