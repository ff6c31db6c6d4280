# round 5 (g): exact-5v5 tests after the precise-softmax change + 5v5 timings; the learner-async GPU tests (stager
# pipeline with zero-copy ring consumption); then the node loop alone (e2e + league_replay) after the ring rework
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_attn_kernels.py "tests/test_exact_mode.py::test_exact_5v5_step_matches_fp64" tests/test_learner_async.py -m gpu > gpurun_out/r5_g_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --model 5v5 --steps 10 --warmup 3 --bf16x3-extra 1 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_5v5x_bench2.json 2> gpurun_out/r5_5v5x_bench2.err || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --bf16x3-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 20 --league-replay-extra 15 --e2e-5v5-extra 15 > gpurun_out/r5_e2e_ring.json 2> gpurun_out/r5_e2e_ring.err
