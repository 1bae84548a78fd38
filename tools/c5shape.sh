#!/bin/bash
# c5 launch shapes (one ring per call vs both rings in one call; one or two
# streams): value, call frac and the call's duration, one bench process each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-c5shape}; mkdir -p $O
for v in "2 1" "1 1" "1 2" "2 1"; do
  set -- $v
  f=$O/c5_p$1_s$2_$(date +%s).log
  timeout -k 10 240 python bench.py --config c5 --rings-per-launch $1 --streams $2 --no-extra --no-cpu-baseline --steps 100 > $f 2>&1 || exit $?
  tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('p=$1 s=$2', d['value'], r['frac'], r['kernel_us_median'], r['frames_per_launch'], d['ms_per_step'])"
done
