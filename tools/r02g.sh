# r02g: batched probes A/B + parity
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02g
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_volume.py -m gpu -q -x --timeout 300 --timeout-method thread -rf -k "config or volume or c5" > gpurun_out/r02g/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r02g/pytest.log
fatal $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
for c in c5 c4; do
  timeout -k 10 400 python tools/abl.py --config $c --rounds 3 --json gpurun_out/r02g/abl_$c.json base nobatch early base@USN_T512=1 nobatch@USN_T512=1 noprobe nosort loadonly > gpurun_out/r02g/abl_$c.log 2>&1
  rc=$?; echo "abl $c rc=$rc"; tail -8 gpurun_out/r02g/abl_$c.log
  fatal $rc && exit $rc
done
timeout -k 10 300 env STAMPS512=1 python tools/stamps.py c5 1048576 > gpurun_out/r02g/stamps_c5.log 2>&1; echo "stamps rc=$?"; tail -12 gpurun_out/r02g/stamps_c5.log
exit 0
