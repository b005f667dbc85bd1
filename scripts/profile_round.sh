#!/bin/bash
# Round profile on one GPU box: rocprofv3 kernel-trace stats of a short bench
# (default schedule + the bench's own serial roofline pass), then PMC passes,
# each counter group in its own run (MI355X_MICROARCH.md "rocprofv3 PMC slots").
# Output under gpurun_out/prof_<tag>/; summaries are copied into profiles/ by hand.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-prover --msm 20,24 --distinct 4096"
SHORT="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prover --msm 20 --no-extras --distinct 4096"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o k -- python3 $BENCH > $OUT/trace.log 2>&1 || { echo "trace run failed"; tail -20 $OUT/trace.log; exit 4; }
tail -c 600 $OUT/trace.log
if [ "${PMC:-1}" = 1 ]; then
  timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/pmc$i -o p -- python3 $SHORT > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/pmc$i.log; exit 5; }
    echo "pmc pass $i ok"
  done
fi
exit 0
