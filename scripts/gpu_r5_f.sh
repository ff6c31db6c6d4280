# round 5 (f): exact 5v5 after the precise-softmax change: its tests, then the 5v5 exact / bf16x3 timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_attn_kernels.py "tests/test_exact_mode.py::test_exact_5v5_step_matches_fp64" -m gpu > gpurun_out/r5_5v5x_tests2.log 2>&1
rc=$?
echo "5v5 exact tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --model 5v5 --steps 10 --warmup 3 --bf16x3-extra 1 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0 > gpurun_out/r5_5v5x_bench2.json 2> gpurun_out/r5_5v5x_bench2.err
