# r02ap: full GPU suite, smoke, bench (512-thread tx, deferred first frame)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02ap
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/r02ap/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU" gpurun_out/r02ap/$name.log | tail -${TAILN:-6}; fatal $rc && exit $rc; return 0; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 5
step rocprof_tx 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02ap/prof_tx -o tx -- python tools/txbench.py 1048576 8 1
exit 0
