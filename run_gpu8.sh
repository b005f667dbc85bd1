set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --msm= --no-prover"
for q in 8 12 16; do
  for i in 3 4 5; do
    GPU_MAX_HW_QUEUES=$q $B --inflight $i > gpurun_out/bench_q${q}_$i.log 2>&1 || exit 1
  done
done
echo EXIT $?
