#!/bin/bash
# c3 launch shapes: queues per step, rings per call and streams (one bench
# process each; the bench's shape is 8 queues in calls of 4 on 2 streams).
#   tools/c3shape.sh [tag]     output: gpurun_out/<tag>/c3_*.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-c3shape}; mkdir -p $O
for v in "8 4 2" "8 2 2" "8 2 4" "16 4 4" "8 4 2" "8 2 2" "8 2 4" "16 4 4"; do
  set -- $v
  f=$O/c3_q$1_p$2_s$3_$(date +%s).log
  timeout -k 10 240 python bench.py --config c3 --queues $1 --rings-per-launch $2 --streams $3 --no-extra --no-cpu-baseline --steps 200 > $f 2>&1 || exit $?
  tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('q=$1 p=$2 s=$3', d['value'], r['frac'], r['kernel_us_median'], r['frames_per_launch'], d['config'].get('enqueue_ms_per_step'), d['ms_per_step'])"
done
