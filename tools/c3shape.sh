set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04al; mkdir -p $O
for v in "8 1" "16 2" "8 2" "16 1"; do
  set -- $v
  timeout -k 10 240 python bench.py --config c3 --queues $1 --streams $2 --no-extra --no-cpu-baseline --steps 200 > $O/c3_q$1_s$2.log 2>&1 || exit $?
  tail -1 $O/c3_q$1_s$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('q=$1 s=$2', d['value'], r['frac'], r['kernel_us_median'], r['frames_per_launch'], d['config'].get('enqueue_ms_per_step'), d['ms_per_step'])"
done
