# learning evidence: GPU learning tests, then the 10-minute learning curve vs the default bot
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_learning.py > gpurun_out/learning_tests.log 2>&1 && \
timeout -k 10 800 python -u scripts/learning_curve.py --budget ${BUDGET:-600} --eval-every 30 --out gpurun_out/r4_learning_curve.jsonl > gpurun_out/learning_curve.log 2>&1
