# r02k: group 10 / load 0.75 image with LDS displacements by default; tx with batched probes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02k
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/r02k/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU" gpurun_out/r02k/$name.log | tail -${TAILN:-9}; fatal $rc && exit $rc; return 0; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step txbench 300 python tools/txbench.py 1048576 12 1
step bench 600 python bench.py --steps 20 --warmup 5
exit 0
