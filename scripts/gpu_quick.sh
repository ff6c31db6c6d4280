# quick loop: exact-kernel numerics + standalone timings
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_exact_mode.py tests/test_gemm_tn.py tests/test_dx_chain.py > gpurun_out/quick_tests.log 2>&1 && \
timeout -k 10 200 python -u scripts/exact_kernels_bench.py > gpurun_out/quick_kbench.log 2>&1
