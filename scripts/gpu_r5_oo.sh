# round 5 (oo): default-priority actor streams — actor GPU tests, then the loops (e2e, config 5, config 4) at the
# 2 s hand-off deadline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_vec_actor.py tests/test_actor_fp8.py tests/test_gpu_runner.py > gpurun_out/r5_oo_tests.log 2>&1 && \
DCA_TEAM_PATIENT=0 timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 20 --e2e-5v5-extra 15 > gpurun_out/r5_oo.json 2> gpurun_out/r5_oo.err
echo "rc=$?"
tail -1 gpurun_out/r5_oo_tests.log
