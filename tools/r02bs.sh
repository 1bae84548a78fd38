# r02bs: tx kernel at 256 vs 512 threads per tile, 1M and 8M-frame rings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bs
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-1} $O/$name.log | cut -c1-300; fatal $rc && exit $rc; return 0; }
for n in 1048576 8388608; do
  step tx512_$n 300 python tools/txbench.py $n 8 1
  USN_TX_T512=0 step tx256_$n 300 python tools/txbench.py $n 8 1
done
exit 0
