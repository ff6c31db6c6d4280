# exact + fp8 numerics (encoder backward in both forms), encoder-backward A/B, actor profiles, the full default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_exact_mode.py tests/test_actor_fp8.py > gpurun_out/round_tests.log 2>&1 && \
DCA_ENC_BWD_X2=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_exact_mode.py > gpurun_out/round_tests_x2.log 2>&1 && \
DCA_ENC_BWD_X2=1 timeout -k 10 200 python -u scripts/exact_kernels_bench.py > gpurun_out/kb_x2.log 2>&1 && \
DCA_ENC_BWD_X2=0 timeout -k 10 200 python -u scripts/exact_kernels_bench.py > gpurun_out/kb_x1.log 2>&1 && \
bash scripts/prof_actor.sh && \
timeout -k 10 700 python -u bench.py > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err
