# r02ac: bench with the probe before the timed steps (20 and 100 steps); every config
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ac
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -v "^\s\|^ Kernel\|^VGPU\|^W20\|^E20" $O/$name.log | tail -${TAILN:-4} | cut -c1-300; fatal $rc && exit $rc; return 0; }
step bench20 600 python bench.py --steps 20 --warmup 5
step bench100 600 python bench.py --steps 100 --warmup 5 --no-extra --no-cpu-baseline
step bench400 600 python bench.py --steps 400 --warmup 5 --no-extra --no-cpu-baseline
TAILN=12 step allcfg 1100 python tools/all_configs.py --out $O/all_configs.json
exit 0
