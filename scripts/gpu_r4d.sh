# actor weight hot-swap (shared operand set per version) numerics + node-loop A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_vec_actor.py tests/test_actor_gpu.py tests/test_actor_fp8.py > gpurun_out/vec_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/e2e_ab.py 15 2048,12,bf16 2048,12,fp8 > gpurun_out/e2e_ab2.log 2> gpurun_out/e2e_ab2.err
