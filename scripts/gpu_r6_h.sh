# round 6 (h): XCD-aware (tile, split) map in the split-K TN GEMM — standalone kernel timings and the learner sections
# of the bench, plain map (DCA_GEMM_XCD=0) vs remap on the same box; the GEMM / exact-mode GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu tests/test_exact_mode.py \
  tests/test_fp32_kernels.py > gpurun_out/r6h_gpu_tests.log 2>&1 || exit $?
DCA_GEMM_XCD=0 timeout -k 10 300 python -u scripts/exact_kernels_bench.py 10 > gpurun_out/r6h_kernels_plain.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/exact_kernels_bench.py 10 > gpurun_out/r6h_kernels_xcd.txt 2>&1 || exit $?
B="--actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0"
DCA_GEMM_XCD=0 timeout -k 10 400 python -u bench.py $B > gpurun_out/r6h_bench_plain.json 2> gpurun_out/r6h_bench_plain.err || exit $?
timeout -k 10 400 python -u bench.py $B > gpurun_out/r6h_bench_xcd.json 2> gpurun_out/r6h_bench_xcd.err || exit $?
DCA_GEMM_XCD=0 timeout -k 10 400 python -u bench.py $B > gpurun_out/r6h_bench_plain2.json 2> gpurun_out/r6h_bench_plain2.err || exit $?
timeout -k 10 400 python -u bench.py $B > gpurun_out/r6h_bench_xcd2.json 2> gpurun_out/r6h_bench_xcd2.err || exit $?
echo done
