# r02bl: tx at larger batches (tiles pipeline once more than the resident 1024): 1M, 2M, 4M, 8M frames
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bl
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20\|tx state\|\"batch\"" $O/$name.log | tail -${TAILN:-4} | cut -c1-400; fatal $rc && exit $rc; return 0; }
for n in 1048576 2097152 4194304 8388608; do
  TAILN=1 step tx_$n 300 python tools/txbench.py $n 8 1
done
exit 0
