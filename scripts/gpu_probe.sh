set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_tn.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gemm_test.log 2>&1 && \
timeout -k 10 300 python -u scripts/gemm_layouts.py > gpurun_out/gemm_layouts.log 2>&1
