# round 5 (final 3): the default bench on the final code
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r5_bench_final3.json 2> gpurun_out/r5_bench_final3.err
echo "rc=$?"
