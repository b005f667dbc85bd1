set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_prover.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/prover_tests.log 2>&1
echo EXIT $?
