# r02ce: registry rehash in parallel regions over a calloc'd table: tx / group / daemon GPU tests, learning rings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ce
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state" $O/$name.log | tail -${TAILN:-4} | cut -c1-200; fatal $rc && exit $rc; return 0; }
step pytest_tx 600 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_group.py tests/test_daemon_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
USN_PROFILE_HOST=1 TAILN=8 step tx_learn_1m 300 python tools/txbench.py 1048576 8 4
grep -E "finalize_tx reserve|^\\{\"batch\"" $O/tx_learn_1m.log | cut -c1-150
exit 0
