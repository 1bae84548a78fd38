set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r02b/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
tail -25 gpurun_out/r02b/pytest.log
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r02b/bench20.json 2> gpurun_out/r02b/bench20.err; echo "bench rc=$?"
tail -c 3000 gpurun_out/r02b/bench20.json; tail -5 gpurun_out/r02b/bench20.err
