# r02bp: counters of the final rx kernel for c5 and c4 (8M frames per launch): HBM traffic
# (FETCH_SIZE / WRITE_SIZE, separate passes), L2 hits/misses, SQ instruction and wait counts
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02bp
mkdir -p $O
export TMPDIR=/tmp
fatal() { [ $1 -ge 124 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
step() { name=$1; to=$2; shift 2; echo "-- $name $(date +%T)"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-2} $O/$name.log | cut -c1-300; fatal $rc && exit $rc; return 0; }
for c in c5 c4; do
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVES"; do
    i=$((i+1))
    rm -rf $O/p_${c}_$i
    step pmc_${c}_$i 120 timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/p_${c}_$i -o run -- python3 tools/kbench.py $c 8388608 12
  done
  TAILN=40 step summary_$c 60 python3 tools/pmc_summary.py $O/p_${c}_1 $O/p_${c}_2 $O/p_${c}_3 $O/p_${c}_4
done
exit 0
