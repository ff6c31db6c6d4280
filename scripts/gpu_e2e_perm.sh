# learner minibatch indices uploaded once per epoch (no per-step host stall): tests + node-loop A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_learner_async.py tests/test_learning.py > gpurun_out/perm_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/e2e_ab.py 15 2048,14,bf16 2048,14,fp8 > gpurun_out/e2e_ab5.log 2> gpurun_out/e2e_ab5.err
