# r02d: probe placement A/B (c4, c5)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02d
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
for c in c5; do
  timeout -k 10 400 python tools/abl.py --config $c --rounds 3 --json gpurun_out/r02d/abl_$c.json base base@USN_PH_GROUP=8 dispglob@USN_PH_GROUP=8 seq seq@USN_PH_GROUP=8 base@USN_PH_LOAD=0.6 base@USN_T512=0 noprobe nosort loadonly > gpurun_out/r02d/abl_$c.log 2>&1
  rc=$?; echo "abl $c rc=$rc"; tail -12 gpurun_out/r02d/abl_$c.log
  fatal $rc && exit $rc
done
exit 0
