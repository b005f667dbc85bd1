#!/bin/bash
# Serial kernel trace (per-kernel durations of one pass) + HBM traffic PMC passes
# of a short serial bench; then the GPU tests + smoke + default bench unless SKIP_CHECK=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03b}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
SHORT="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-prover --no-seam --no-ppb --msm 20 --distinct 4096 --serial --slots 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o k -- python3 $SHORT > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 4; }
echo "trace ok"
if [ "${PMC:-1}" = 1 ]; then
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES"; do
    i=$((i + 1))
    timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/pmc$i -o p -- python3 $SHORT > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/pmc$i.log; exit 5; }
    echo "pmc pass $i ok"
  done
fi
if [ "${SKIP_CHECK:-0}" != 1 ]; then
  bash scripts/gpu_check.sh || exit $?
fi
exit 0
