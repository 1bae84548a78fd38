# r02h: A/B of batched probes (1M and 8M launches), tx timing, host loop, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02h
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/r02h/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU" gpurun_out/r02h/$name.log | tail -${TAILN:-9}; fatal $rc && exit $rc; return 0; }
step abl_c5 400 python tools/abl.py --config c5 --rounds 3 base nobatch early noprobe nosort
step abl_c4 400 python tools/abl.py --config c4 --rounds 3 base nobatch base@USN_T512=1 noprobe nosort
step abl_c5_8m 400 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 3 --launches 30 base nobatch noprobe nosort
step txbench 300 python tools/txbench.py 1048576 12 1
step hostio 300 python tools/hostio.py c2 1048576 8 4 6
step bench 600 python bench.py --steps 20 --warmup 5
step abl_c5_lo 300 python tools/abl.py --config c5 --rounds 3 base loadonly
exit 0
