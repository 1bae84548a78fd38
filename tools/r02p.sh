# r02p: tx one launch, tiles by block index (no ticket atomics)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02p
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; timeout -k 10 $to "$@" > gpurun_out/r02p/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU" gpurun_out/r02p/$name.log | tail -${TAILN:-12}; fatal $rc && exit $rc; return 0; }
step pytest_tx 400 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_group.py -x -q --timeout 120 --timeout-method thread
step txbench 200 python tools/txbench.py 1048576 12 1
step txbench4 200 python tools/txbench.py 1048576 12 4
rm -rf gpurun_out/r02p/txprof
step txprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02p/txprof -o run -- python3 tools/txbench.py 1048576 24 1
python3 tools/trace_summary.py gpurun_out/r02p/txprof/run_kernel_trace.csv
step txstamps 200 python tools/stamps.py c4tx 1048576
exit 0
