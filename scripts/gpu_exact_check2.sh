set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/exact_kernels_bench.py > gpurun_out/exact_kbench.log 2>&1 && \
DCA_EXACT_ACT=fast timeout -k 10 300 python -u -m pytest -x -s --timeout 300 --timeout-method thread tests/test_exact_mode.py -k deploy > gpurun_out/exact_fast_act.log 2>&1 ; \
DCA_EXACT_ACT=libm timeout -k 10 300 python -u -m pytest -x -s --timeout 300 --timeout-method thread tests/test_exact_mode.py -k deploy > gpurun_out/exact_libm_act.log 2>&1 ; \
DCA_EXACT_ACT=fast timeout -k 10 300 python -u bench.py --precision fp32-exact --steps 20 --warmup 5 --actor 0 --e2e 0 --bf16x3-extra 0 --model-5v5-extra 0 > gpurun_out/exact_fast_bench.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fused_policy.py tests/test_learner_async.py tests/test_optim.py -m gpu > gpurun_out/fused_tests.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_packing.py tests/test_lstm_kernel.py -m gpu > gpurun_out/packing_tests.log 2>&1
timeout -k 10 400 python -u scripts/learning_curve.py --budget 60 --eval-every 20 --eval-games 64 --out gpurun_out/curve_smoke.jsonl > gpurun_out/curve_smoke.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_actor_fp8.py tests/test_actor_gpu.py tests/test_vec_actor.py -m gpu > gpurun_out/actor_tests.log 2>&1
