# round 6 (w): reset flags compared at their use (lstm_team.hip) — probe, packing/exact tests, e2e with the actor
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/reset_probe.py 10 > gpurun_out/r6w_reset_probe.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_packing.py tests/test_exact_mode.py > gpurun_out/r6w_tests.log 2>&1 || exit $?
E="--bf16x3-extra 0 --vtrace-extra 0 --model-5v5-extra 0 --model-5v5-exact-extra 0 --bptt350-extra 0 --big-batch-extra 0 --actor 0 --league-replay-extra 0 --e2e-5v5-extra 0 --e2e-extra 0"
timeout -k 10 300 python -u bench.py $E > gpurun_out/r6w_e2e.json 2> gpurun_out/r6w_e2e.err || exit $?
echo done
