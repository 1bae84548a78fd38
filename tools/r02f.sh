# r02f: phase stamps per config
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02f
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
run() { name=$1; shift; timeout -k 10 300 env "$@" > gpurun_out/r02f/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; cat gpurun_out/r02f/$name.log | tail -12; fatal $rc && exit $rc; return 0; }
run c5_512 STAMPS512=1 python tools/stamps.py c5 1048576
run c5_256 USN_T512=0 python tools/stamps.py c5 1048576
run c4 python tools/stamps.py c4 1048576
run c2 STAMPS512=1 python tools/stamps.py c2 1048576
exit 0
