set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in 0 1 2; do
  FTZ_G1_AFTER=$a timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --msm '' --no-prover > gpurun_out/bench_after$a.log 2>&1 || exit 1
done
echo EXIT $?
