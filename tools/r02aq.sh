# r02aq: bench at 20 steps vs the ramp length (40 / 100 / 200 untimed rounds each side of the probe), and 400 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02aq
mkdir -p $O
run() {
  local tag=$1; shift
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-extra "$@" > $O/$tag.json 2> $O/$tag.err || exit 1
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_us_median'])"
}
run r40_a --steps 20 --warmup 5 --ramp 40
run r100_a --steps 20 --warmup 5 --ramp 100
run r200_a --steps 20 --warmup 5 --ramp 200
run r40_b --steps 20 --warmup 5 --ramp 40
run r100_b --steps 20 --warmup 5 --ramp 100
run r200_b --steps 20 --warmup 5 --ramp 200
run s400 --steps 400 --warmup 5 --ramp 40
