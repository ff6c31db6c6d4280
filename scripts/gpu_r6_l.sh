# round 6 (l): final full bench (driver defaults)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r6l_bench.json 2> gpurun_out/r6l_bench.err || exit $?
echo done
