# actor-step numerics (bf16 + fp8) and the two actor kernel profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_actor_fp8.py tests/test_actor_gpu.py > gpurun_out/actor_tests.log 2>&1 && \
bash scripts/prof_actor.sh && \
timeout -k 10 300 python -u scripts/actor_bench.py 2048 bf16 > gpurun_out/ab_bf16.log 2>&1 && \
timeout -k 10 300 python -u scripts/actor_bench.py 2048 fp8 > gpurun_out/ab_fp8.log 2>&1
