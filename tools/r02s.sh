# r02s: full GPU suite, smoke, bench on the one-launch tx tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02s
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/r02s/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU" gpurun_out/r02s/$name.log | tail -${TAILN:-6}; fatal $rc && exit $rc; return 0; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 5
exit 0
