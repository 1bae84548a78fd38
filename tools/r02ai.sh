# r02ai: tx without probes (bound), bench after persistence revert
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ai
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20" $O/$name.log | tail -${TAILN:-8}; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc; return 0; }
TAILN=3 step tx_base 200 python tools/txbench.py 1048576 8 1
TAILN=3 step tx_noprobe 200 python tools/txbench.py 1048576 8 1 build/abl/txnoprobe/libusn.so
step bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
exit 0
