# exact-fp32 kernels: numerics tests, then a kernel profile of the exact learner step (results under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gemm_tn.py tests/test_exact_mode.py tests/test_dx_chain.py > gpurun_out/exact_tests.log 2>&1 && \
bash scripts/prof_exact.sh ${1:-profx1}
