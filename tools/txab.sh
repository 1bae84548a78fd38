#!/bin/bash
# tx A/B: tools/txbench.py on the in-tree library and on A/B builds, interleaved
# (rotating buffers, 24 rings): tools/txab.sh TAG variant...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; shift; mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    L=build/abl/$v/libusn.so
    timeout -k 10 120 python tools/txbench.py 1048576 24 1 $L --rotate 6 > $O/tx_${v}_$rep.log 2>&1 || exit $?
    echo "$v $(tail -1 $O/tx_${v}_$rep.log | cut -c1-300)"
  done
done
