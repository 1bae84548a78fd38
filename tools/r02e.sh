# r02e: late header DMA A/B + GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02e
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
for c in c5 c4; do
  timeout -k 10 400 python tools/abl.py --config $c --rounds 3 --json gpurun_out/r02e/abl_$c.json base dispglob early base@USN_PH_GROUP=4 noprobe nosort loadonly > gpurun_out/r02e/abl_$c.log 2>&1
  rc=$?; echo "abl $c rc=$rc"; tail -7 gpurun_out/r02e/abl_$c.log
  fatal $rc && exit $rc
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_group.py -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r02e/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r02e/pytest.log
exit 0
