#!/bin/bash
# LDS instructions and bank-conflict cycles per kernel for library builds
# (short bench, one PMC pass each); LIBS as scripts/ab_lib.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHORT="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prover --msm= --no-seam --no-ppb --no-extras --distinct 4096"
IFS='|' read -ra SETS <<< "${LIBS:-}"
for s in "${SETS[@]}"; do
  name=${s%%=*}; path=${s#*=}
  if [ "$path" = "default" ]; then lib=""; else lib="--lib $PWD/$path"; fi
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES -d gpurun_out/pmclds_$name -o p -- python3 $SHORT $lib > gpurun_out/pmclds_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/pmclds_$name.log; exit 5; }
  echo "pmc $name ok"
done
