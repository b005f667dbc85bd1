#!/bin/bash
# PMC VALU count per kernel for two libraries (short bench), one pass each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHORT="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prover --msm= --no-seam --no-ppb --no-extras --distinct 4096"
IFS='|' read -ra SETS <<< "${LIBS:-}"
for s in "${SETS[@]}"; do
  name=${s%%=*}; path=${s#*=}
  if [ "$path" = "default" ]; then lib=""; else lib="--lib $PWD/$path"; fi
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmcab_$name -o p -- python3 $SHORT $lib > gpurun_out/pmcab_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/pmcab_$name.log; exit 5; }
  echo "pmc $name ok"
done
