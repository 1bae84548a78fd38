#!/bin/bash
# bench variants: rx queues / streams per GPU for c5 (20 and 200 steps)
set -o pipefail
mkdir -p gpurun_out/r02ag
cd "$GRAFT_REPO_ROOT" || exit 1
run() {
  local tag=$1; shift
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-extra "$@" > gpurun_out/r02ag/$tag.json 2> gpurun_out/r02ag/$tag.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/r02ag/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_us_median'], d['config']['rx_queues_per_gpu'], d['config']['streams'])"
}
run q2s2_20 --steps 20 --warmup 5
run q2s2_200 --steps 200 --warmup 5
run q4s2_20 --steps 20 --warmup 5 --queues 4
run q4s2_200 --steps 200 --warmup 5 --queues 4
run q4s4_20 --steps 20 --warmup 5 --queues 4 --streams 4
run q3s3_20 --steps 20 --warmup 5 --queues 3 --streams 3
run q3s3_200 --steps 200 --warmup 5 --queues 3 --streams 3
