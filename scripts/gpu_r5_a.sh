# round 5: actor core tests, exact-path tests (multi-row chains, compat network), then the half-team probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_actor_gpu.py tests/test_actor_fp8.py -m gpu > gpurun_out/r5_actor_tests.log 2>&1
rc=$?
echo "actor tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_exact_mode.py tests/test_optim.py -m gpu > gpurun_out/r5_exact_tests.log 2>&1
rc=$?
echo "exact tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_r5_half.sh
