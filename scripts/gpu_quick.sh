# quick loop: exact-kernel numerics + standalone timings + the headline step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_exact_mode.py tests/test_gemm_tn.py tests/test_dx_chain.py tests/test_packing.py > gpurun_out/quick_tests.log 2>&1 && \
timeout -k 10 200 python -u scripts/exact_kernels_bench.py > gpurun_out/quick_kbench.log 2>&1 && \
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --bf16x3-extra 0 --model-5v5-extra 0 --actor 0 --e2e 0 > gpurun_out/quick_bench.log 2> gpurun_out/quick_bench.err
