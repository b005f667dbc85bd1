set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="timeout -k 10 200 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --msm= --no-prover"
for q in 8 12 16; do
  for i in 3 4 5 6; do
    GPU_MAX_HW_QUEUES=$q $B --inflight $i > gpurun_out/bench_q${q}_$i.log 2>&1 || exit 1
  done
done
for f in gpurun_out/bench_q*.log; do echo $f; tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["batch_latency_ms"])"; done
echo EXIT 0
