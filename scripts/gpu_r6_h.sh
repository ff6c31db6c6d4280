# round 6 (h): XCD-aware (tile, split) map in the split-K TN GEMM (DCA_GEMM_XCD) and the balanced 5v5 weight-gradient
# streams (DCA_5V5_WG_BALANCE) — standalone kernel timings and the learner sections of the bench, on one box,
# baseline (both off) first and last; the GEMM / exact-mode GPU tests (with the 5v5 worst-tensor print)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu tests/test_exact_mode.py \
  tests/test_fp32_kernels.py > gpurun_out/r6h_gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_featurize.py \
  tests/test_vec_actor.py > gpurun_out/r6h_gpu_tests_featurize.log 2>&1 || exit $?
for P in bf16 fp8; do
  timeout -k 10 300 python -u scripts/actor_bench.py 2048 $P > gpurun_out/r6h_actor_$P.json 2>&1 || exit $?
done
DCA_GEMM_XCD=0 timeout -k 10 300 python -u scripts/exact_kernels_bench.py 10 > gpurun_out/r6h_kernels_plain.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/exact_kernels_bench.py 10 > gpurun_out/r6h_kernels_xcd.txt 2>&1 || exit $?
B="--actor 0 --e2e 0 --league-replay-extra 0 --e2e-5v5-extra 0"
run() {  # name xcd balance
  DCA_GEMM_XCD=$2 DCA_5V5_WG_BALANCE=$3 timeout -k 10 400 python -u bench.py $B > gpurun_out/r6h_bench_$1.json 2> gpurun_out/r6h_bench_$1.err
}
run base 0 0 && run xcd 1 0 && run both 1 1 && run bal 0 1 && run base2 0 0 && run both2 1 1 || exit $?
echo done
