cd $GRAFT_REPO_ROOT
for s in 4 6 4 6 5 8; do
  timeout -k 10 120 python -u bench.py --steps 60 --warmup 2 --msm "" --no-cpu-baseline --no-prover --no-extras --slots $s > gpurun_out/s.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/s.json')); print($s, d['value'], d['engine'])"
done
