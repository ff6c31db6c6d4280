# ingest with blocking slot events: numerics + node-loop A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_learner_async.py > gpurun_out/ingest_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/e2e_ab.py 15 2048,12,bf16 2048,12,fp8 > gpurun_out/e2e_ab3.log 2> gpurun_out/e2e_ab3.err
