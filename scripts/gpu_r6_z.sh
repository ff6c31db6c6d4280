# round 6 (z): shared-GPU two-rank rehearsal (patient hand-off deadline) + final full bench (driver defaults)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 650 --timeout-method thread -m gpu tests/test_bench_gpu_dist.py > gpurun_out/r6z_dist.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/r6z_bench.json 2> gpurun_out/r6z_bench.err || exit $?
echo done
