# round 5: the whole GPU test suite without stopping at the first failure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r5_gpu_tests_all.log 2>&1
echo "tests rc=$?"
tail -15 gpurun_out/r5_gpu_tests_all.log
