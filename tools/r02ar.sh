# r02ar: keys per displacement group (USN_PH_GROUP 10 / 12 / 16 / 20) at c5 8M; 2-rank bench rehearsal on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ar
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20" $O/$name.log | tail -${TAILN:-8}; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc; return 0; }
step abl_group 600 python tools/abl.py --config c5 --frames 8388608 --batches 2 --rounds 3 --launches 30 base base@USN_PH_GROUP=12 base@USN_PH_GROUP=16 base@USN_PH_GROUP=20
TAILN=2 step bench_n2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline
TAILN=2 step bench_n2_strong 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --strong
exit 0
