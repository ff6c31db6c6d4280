# round 5 (final 2): whole GPU test suite + smoke, then the default bench, on the final code
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r5_final2_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_final2_smoke.log 2>&1 && \
timeout -k 10 900 python -u bench.py > gpurun_out/r5_bench_final2.json 2> gpurun_out/r5_bench_final2.err
echo "rc=$?"
tail -1 gpurun_out/r5_final2_tests.log; tail -1 gpurun_out/r5_final2_smoke.log
