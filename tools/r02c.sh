# r02c: GPU tests on the perfect-hash image, A/B old (r01 kernel) vs new per config, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02c
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r02c/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r02c/pytest.log
fatal $rc && exit $rc
for c in c2 c3 c4 c5; do
  timeout -k 10 300 python tools/abl.py --config $c --rounds 3 --json gpurun_out/r02c/abl_$c.json old base noprobe nosort loadonly > gpurun_out/r02c/abl_$c.log 2>&1
  rc=$?; echo "abl $c rc=$rc"; tail -6 gpurun_out/r02c/abl_$c.log
  fatal $rc && exit $rc
done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r02c/bench20.json 2> gpurun_out/r02c/bench20.err; echo "bench rc=$?"
tail -c 4000 gpurun_out/r02c/bench20.json; tail -5 gpurun_out/r02c/bench20.err
