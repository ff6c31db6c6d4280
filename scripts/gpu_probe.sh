set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_policy.py -x -v -k "rccl or graph" --timeout 200 --timeout-method thread > gpurun_out/pg_test.log 2>&1
