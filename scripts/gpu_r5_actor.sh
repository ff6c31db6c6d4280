set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_actor_gpu.py tests/test_actor_fp8.py -m gpu > gpurun_out/r5_actor_tests.log 2>&1
